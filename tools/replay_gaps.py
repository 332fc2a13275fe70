"""Per-replay timing of the learner step's HIP graph from a rocprofv3 kernel trace: where the time between kernels goes.

    python tools/replay_gaps.py <kernel_trace.csv> [--marker FusedAdam] [--skip 3] [--count 20]

Steps are delimited by the marker kernel (Adam, the last launch of a step).  --skip drops the first markers (the
capture's three eager warm-up steps run before the first replay); --count replays follow.  For each replay:
  period   = end of its last kernel - end of the previous step's last kernel (what the bench's clock sees per step);
  kernels  = sum of its kernel durations;
  gaps     = start of kernel k+1 - end of kernel k inside the step (dispatch / dependency latency), and the gap
             between the previous step's marker and this step's first kernel (the replay boundary).
Prints per-replay rows, the mean over the replays, and for the median replay each kernel with the gap before it.
"""
import csv
import statistics
import sys


def short(name):
    return name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:90]


def main():
    path = sys.argv[1]
    opt = lambda k, d: type(d)(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else d   # noqa: E731
    marker, skip, count = opt('--marker', 'FusedAdam'), opt('--skip', 3), opt('--count', 20)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    steps = []
    for j in range(skip, min(skip + count, len(ends))):
        lo, hi = ends[j - 1] + 1, ends[j] + 1
        ks = rows[lo:hi]
        st = [int(r['Start_Timestamp']) for r in ks]
        en = [int(r['End_Timestamp']) for r in ks]
        prev_end = int(rows[ends[j - 1]]['End_Timestamp'])
        dur = [(e - s) / 1e3 for s, e in zip(st, en)]
        gaps = [(st[0] - prev_end) / 1e3] + [(st[k + 1] - en[k]) / 1e3 for k in range(len(ks) - 1)]
        steps.append({'period': (en[-1] - prev_end) / 1e3, 'kernels': sum(dur), 'n': len(ks), 'gaps': gaps,
                      'dur': dur, 'names': [short(r['Kernel_Name']) for r in ks],
                      'overlap': sum(-g for g in gaps if g < 0)})
    if not steps:
        raise SystemExit('no complete steps between markers %r' % marker)
    print('%6s %9s %9s %9s %9s %9s %6s' % ('replay', 'period', 'kernels', 'gap_sum', 'gap_max', 'boundary', 'n'))
    for i, s in enumerate(steps):
        pos = [g for g in s['gaps'] if g > 0]
        print('%6d %9.2f %9.2f %9.2f %9.2f %9.2f %6d' % (i, s['period'], s['kernels'], sum(pos), max(pos),
                                                          s['gaps'][0], s['n']))
    mean = lambda k: statistics.mean(s[k] for s in steps)   # noqa: E731
    gsum = statistics.mean(sum(g for g in s['gaps'] if g > 0) for s in steps)
    print('mean over %d replays: period %.2f us, kernels %.2f us, positive gaps %.2f us (%.1f%% of the period), '
          '%d kernels, %.2f us per boundary' % (len(steps), mean('period'), mean('kernels'), gsum,
                                               100 * gsum / mean('period'), steps[0]['n'],
                                               gsum / max(steps[0]['n'], 1)))
    med = sorted(steps, key=lambda s: s['period'])[len(steps) // 2]
    print('\nmedian replay (period %.2f us): gap before each kernel, its duration' % med['period'])
    for g, d, n in zip(med['gaps'], med['dur'], med['names']):
        print('%8.2f %8.2f  %s' % (g, d, n))


if __name__ == '__main__':
    main()
