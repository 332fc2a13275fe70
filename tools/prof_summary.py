"""Summarise a rocprofv3 kernel trace (CSV) per learner step.

    python tools/prof_summary.py <run_kernel_trace.csv> <steps> [--match NAME]
<steps> may be 'per:SUBSTR': the number of launches of the (once-per-step)
kernel whose name contains SUBSTR, e.g. per:fused_adam.
Prints kernel-name groups with total time per step and mean duration per call.
"""
import collections
import csv
import sys


def main():
    path, steps = sys.argv[1], sys.argv[2]
    match = sys.argv[sys.argv.index('--match') + 1] if '--match' in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    if steps.startswith('per:'):
        steps = sum(1 for r in rows if steps[4:] in r['Kernel_Name'])
    steps = int(steps)
    tot, cnt = collections.Counter(), collections.Counter()
    for r in rows:
        n = r['Kernel_Name']
        if match and match not in n:
            continue
        n = n.replace('(anonymous namespace)::', '').replace('void ', '')
        n = n.split('(')[0][:110]
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        tot[n] += d
        cnt[n] += 1
    total = sum(tot.values())
    print('| us/step | calls | mean us | share | kernel |')
    print('|---:|---:|---:|---:|---|')
    for n, t in tot.most_common(30):
        print('| %.1f | %d | %.2f | %.1f%% | `%s` |' % (t / 1e3 / steps, cnt[n], t / 1e3 / cnt[n], 100 * t / total, n))
    print('\ntotal kernel time %.3f ms/step over %d steps' % (total / 1e6 / steps, steps))


if __name__ == '__main__':
    main()
