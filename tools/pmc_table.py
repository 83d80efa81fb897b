"""Median per-dispatch counter values of one kernel from rocprofv3 --pmc CSV directories.
usage: pmc_table.py KERNEL_SUBSTRING DIR..."""
import csv
import glob
import statistics
import sys

kern = sys.argv[1]
for d in sys.argv[2:]:
    by = {}
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if kern not in r['Kernel_Name']:
                continue
            by.setdefault(r['Counter_Name'], {}).setdefault(r['Dispatch_Id'], 0.0)
            by[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
    med = {k: statistics.median(v.values()) for k, v in by.items()}
    print(d, ' '.join(f'{k}={med[k]/1e6:.2f}M' for k in sorted(med)))
