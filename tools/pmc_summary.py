"""Per-dispatch PMC values for kernels matching a name, from rocprofv3 counter_collection.csv."""
import csv, sys, collections
path, match = sys.argv[1], sys.argv[2]
rows = [r for r in csv.DictReader(open(path)) if match in r['Kernel_Name']]
by = collections.defaultdict(dict)
for r in rows:
    by[(r['Dispatch_Id'], r['Grid_Size'] if 'Grid_Size' in r else '')][r['Counter_Name']] = float(r['Counter_Value'])
for (d, gs), c in sorted(by.items(), key=lambda kv: int(kv[0][0])):
    print(d, gs, c)
