"""Print the ordered kernel sequence of one learner step from a rocprofv3 kernel trace.

    python tools/step_sequence.py <kernel_trace.csv> [--marker fused_adam] [--index -2]
Steps are delimited by the marker kernel (one per step); prints name and duration.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[sys.argv.index('--marker') + 1] if '--marker' in sys.argv else 'FusedAdam'
    index = int(sys.argv[sys.argv.index('--index') + 1]) if '--index' in sys.argv else -2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    lo, hi = ends[index - 1] + 1, ends[index] + 1
    tot = 0
    for r in rows[lo:hi]:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        tot += d
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:100]
        print('%8.2f  %s' % (d, n))
    print('%8.2f  total kernel us, %d kernels' % (tot, hi - lo))


if __name__ == '__main__':
    main()
