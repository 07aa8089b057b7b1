"""Top kernels of a rocprofv3 kernel_stats.csv: python tools/kstat_top.py file.csv [n]"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print(f"{float(x['TotalDurationNs']) / 1e6:8.2f} ms {x['Calls']:>5} {float(x['AverageNs']) / 1e3:9.1f} us  {x['Name'][:100]}")
