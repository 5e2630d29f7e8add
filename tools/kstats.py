"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, %)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:64]:64s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:10.1f}us "
          f"{float(r['Percentage']):6.2f}%")
