"""HBM bytes per launch of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), gfx950-corrected.

    python tools/pmc_bytes.py KERNEL_SUBSTRING ALGORITHMIC_BYTES FETCH.csv WRITE.csv [--skip N] [--label TEXT]

Per MI355X_MICROARCH.md (HBM / rocprofv3) gfx950's FETCH_SIZE counts half the bytes of a wide coalesced streaming
read: read bytes = 2 x FETCH_SIZE x 1024, write bytes = WRITE_SIZE x 1024.  Dispatches are averaged after skipping the
first N of the kernel (warm-up).  One JSON object on stdout (the layout of profiles/r04_block_pmc.json).
"""
import argparse
import csv
import json


def per_dispatch(path, kernel, counter):
    by = {}
    for r in csv.DictReader(open(path)):
        if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter:
            d = int(r['Dispatch_Id'])
            by[d] = by.get(d, 0.0) + float(r['Counter_Value'])
    return [by[d] for d in sorted(by)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('kernel')
    ap.add_argument('algorithmic', type=int)
    ap.add_argument('fetch')
    ap.add_argument('write')
    ap.add_argument('--skip', type=int, default=2)
    ap.add_argument('--label', default='')
    o = ap.parse_args()
    f = per_dispatch(o.fetch, o.kernel, 'FETCH_SIZE')[o.skip:]
    w = per_dispatch(o.write, o.kernel, 'WRITE_SIZE')[o.skip:]
    fetch, write = sum(f) / len(f), sum(w) / len(w)
    rb, wb = int(2 * fetch * 1024), int(write * 1024)
    print(json.dumps({'kernel': o.kernel, 'label': o.label, 'dispatches': [len(f), len(w)],
                      'FETCH_SIZE_KB': round(fetch, 1), 'WRITE_SIZE_KB': round(write, 1),
                      'read_bytes_corrected': rb, 'write_bytes': wb, 'bytes_per_launch': rb + wb,
                      'algorithmic_bytes': o.algorithmic,
                      'traffic_over_algorithmic': round((rb + wb) / o.algorithmic, 3)}, indent=1))


if __name__ == '__main__':
    main()
