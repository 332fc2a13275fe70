"""The scan's PMC traffic per launch size from the FETCH_SIZE / WRITE_SIZE passes over tools/scan_pmc.py (launches
grouped by grid size: B=4096 T=32 and the cold B=2^18 T=32), in the layout of profiles/r03s4_scan_pmc.json.

    python tools/scan_pmc_json.py FETCH.csv WRITE.csv > profiles/r06_scan_pmc.json
"""
import csv
import json
import sys

KERNEL = 'targets_kernel'
SIZES = {4096: False, 1 << 18: True}     # B -> cold


def by_grid(path, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r['Kernel_Name'] and r['Counter_Name'] == counter:
            key = (int(r['Grid_Size']), int(r['Dispatch_Id']))
            per[key] = per.get(key, 0.0) + float(r['Counter_Value'])
    out = {}
    for (grid, _), v in sorted(per.items()):
        out.setdefault(grid, []).append(v)
    return {g: sum(v) / len(v) for g, v in out.items()}


def main():
    f, w = by_grid(sys.argv[1], 'FETCH_SIZE'), by_grid(sys.argv[2], 'WRITE_SIZE')
    grids = sorted(f)
    configs = []
    for (B, cold), grid in zip(sorted(SIZES.items()), grids):
        T, P, Pp = 32, 2, 1
        alg = B * T * (4 * P + 4 * Pp + 4 * Pp + 4 * P + 4 * P) + B * 4 * P   # values, rho, c, targets, adv + returns
        rb, wb = int(2 * f[grid] * 1024), int(w[grid] * 1024)
        c = {'B': B, 'T': T, 'grid_threads': grid, 'fetch_size_kb': round(f[grid], 2),
             'write_size_kb': round(w[grid], 2), 'read_bytes': rb, 'write_bytes': wb, 'traffic_bytes': rb + wb,
             'algorithmic_bytes': alg, 'traffic_over_algorithmic': round((rb + wb) / alg, 3)}
        if cold:
            c['cold'] = True
        configs.append(c)
    print(json.dumps({'kernel': 'targets_kernel<VTRACE,UPGO,REW=0,RETT=0> (hrl_compute_targets_fused, value head)',
                      'round': 'r06 (final tree)',
                      'source': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes over '
                                'tools/scan_pmc.py; per-dispatch values averaged per launch size',
                      'correction': 'gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read '
                                    '(MI355X_MICROARCH.md HBM): read bytes = 2 * FETCH_SIZE * 1024; write bytes = '
                                    'WRITE_SIZE * 1024',
                      'configs': configs}, indent=1))


if __name__ == '__main__':
    main()
