"""HBM traffic of the chain block backward from two rocprofv3 PMC passes over tools/block_bench.py.

    python tools/block_pmc.py FETCH_counter_collection.csv WRITE_counter_collection.csv > profiles/r03_block_pmc.json

Averages FETCH_SIZE and WRITE_SIZE (KB) over the conv3x3_block_bwd2_kernel dispatches.  Per MI355X_MICROARCH.md
(HBM / rocprofv3) gfx950's FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so the corrected
read bytes are 2 x FETCH_SIZE; the kernel's loads are 12- and 8-byte runs per lane, so the raw counter is kept
beside the corrected figure.  bytes_per_launch = 2 x FETCH + WRITE.
"""
import csv
import json
import sys

KERNEL = 'conv3x3_block_bwd2_kernel'


def mean_counter(path, name):
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if KERNEL in r['Kernel_Name'] and r['Counter_Name'] == name]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch, nf = mean_counter(sys.argv[1], 'FETCH_SIZE')
    write, nw = mean_counter(sys.argv[2], 'WRITE_SIZE')
    M = 131072
    algorithmic = 4 * M * 288 * 4
    out = {'kernel': KERNEL, 'M': M, 'dispatches': [nf, nw], 'FETCH_SIZE_KB': round(fetch, 1),
           'WRITE_SIZE_KB': round(write, 1), 'read_bytes_corrected': int(2 * fetch * 1024),
           'write_bytes': int(write * 1024), 'bytes_per_launch': int(2 * fetch * 1024 + write * 1024),
           'algorithmic_bytes': algorithmic,
           'traffic_over_algorithmic': round((2 * fetch * 1024 + write * 1024) / algorithmic, 3)}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
