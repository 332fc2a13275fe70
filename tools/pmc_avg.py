"""Mean per dispatch of every counter for kernels matching a name (rocprofv3 counter_collection.csv), skipping
the first two dispatches (warm-up)."""
import collections
import csv
import sys

path, match = sys.argv[1], sys.argv[2]
by = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(path)):
    if match not in r['Kernel_Name']:
        continue
    d = int(r['Dispatch_Id'])
    by[d][r['Counter_Name']] = by[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    names[d] = r['Kernel_Name'][:80]
ds = sorted(by)[2:] or sorted(by)
tot = collections.defaultdict(float)
for d in ds:
    for k, v in by[d].items():
        tot[k] += v
print(names[ds[0]] if ds else '-', len(ds), {k: round(v / len(ds), 1) for k, v in sorted(tot.items())})
