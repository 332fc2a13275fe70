"""Sum rocprofv3 PMC counters per kernel from a rocpd database (rocprofv3 --pmc ... -d DIR -o NAME).

    python tools/pmc_db.py gpurun_out/.../pmc_results.db [substring]
Prints, per kernel name containing `substring`, the dispatch count and each counter summed per dispatch
(mean over dispatches).
"""
import collections
import sqlite3
import sys


def main():
    db, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else '')
    c = sqlite3.connect(db)
    rows = c.execute('select dispatch_id, kernel_name, counter_name, value from counters_collection').fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for d, k, n, v in rows:
        if sub in k:
            per[d][n] += v
            names[d] = k
    by_kernel = collections.defaultdict(list)
    for d, cnt in per.items():
        by_kernel[names[d][:90]].append(cnt)
    for k, lst in by_kernel.items():
        keys = sorted(lst[0])
        print('%s  (%d dispatches)' % (k, len(lst)))
        for n in keys:
            print('   %-28s %16.0f' % (n, sum(x[n] for x in lst) / len(lst)))


if __name__ == '__main__':
    main()
