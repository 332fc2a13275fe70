"""Per-kernel durations of early vs late graph replays in a rocprofv3 kernel trace (why the first replays after a
capture run slow): replays are delimited by the marker kernel as in tools/replay_gaps.py.

    python tools/replay_kernels.py <kernel_trace.csv> [--marker adam_clip_kernel] [--skip 3] [--early 0:5] [--late 40:45]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    opt = lambda k, d: type(d)(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else d   # noqa: E731
    marker, skip = opt('--marker', 'adam_clip_kernel'), opt('--skip', 3)
    early = [int(v) for v in opt('--early', '0:5').split(':')]
    late = [int(v) for v in opt('--late', '40:45').split(':')]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    reps = []
    for j in range(skip + 1, len(ends)):
        reps.append(rows[ends[j - 1] + 1:ends[j] + 1])

    def mean_of(lo, hi):
        sel = reps[lo:hi]
        n = min(len(r) for r in sel)
        out = []
        for k in range(n):
            d = [(int(r[k]['End_Timestamp']) - int(r[k]['Start_Timestamp'])) / 1e3 for r in sel]
            out.append((sel[0][k]['Kernel_Name'], sum(d) / len(d)))
        per = [(int(r[-1]['End_Timestamp']) - int(r[0]['Start_Timestamp'])) / 1e3 for r in sel]
        return out, sum(per) / len(per)

    a, pa = mean_of(*early)
    b, pb = mean_of(*late)
    print('replays %d..%d: period %.2f us; replays %d..%d: period %.2f us (of %d replays)' %
          (early[0], early[1] - 1, pa, late[0], late[1] - 1, pb, len(reps)))
    print('%10s %10s %8s  kernel' % ('early_us', 'late_us', 'ratio'))
    for (n, x), (_, y) in zip(a, b):
        name = n.split('(')[0].replace('void ', '').replace('(anonymous namespace)::', '')[:70]
        print('%10.2f %10.2f %8.3f  %s' % (x, y, x / y if y else 0.0, name))


if __name__ == '__main__':
    main()
