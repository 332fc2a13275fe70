"""Mean duration of one kernel per launch grid, from a rocprofv3 kernel trace (CSV).

    python tools/kernel_by_grid.py <kernel_trace.csv> <name substring>
Separates e.g. the learner step's own scan launch from the bench's hot/cold scan timing launches.
"""
import collections
import csv
import sys


def main():
    path, match = sys.argv[1], sys.argv[2]
    tot, cnt, names = collections.Counter(), collections.Counter(), {}
    for r in csv.DictReader(open(path)):
        if match not in r['Kernel_Name']:
            continue
        key = (r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0],
               r.get('Grid_Size_X', r.get('Grid_Size', '?')), r.get('LDS_Block_Size', r.get('Lds_Size', '?')))
        tot[key] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        cnt[key] += 1
    print('| kernel | grid x | LDS | launches | mean us |')
    print('|---|---:|---:|---:|---:|')
    for key in sorted(tot, key=lambda k: -cnt[k]):
        print('| `%s` | %s | %s | %d | %.2f |' % (key[0], key[1], key[2], cnt[key], tot[key] / 1e3 / cnt[key]))


if __name__ == '__main__':
    main()
