"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, %).
Optional further arguments keep only kernels whose name contains one of them."""
import csv
import sys

keep = sys.argv[2:]
for r in csv.DictReader(open(sys.argv[1])):
    if keep and not any(k in r["Name"] for k in keep):
        continue
    print(f"{r['Name'][:64]:64s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:10.1f}us "
          f"{float(r['Percentage']):6.2f}%")
