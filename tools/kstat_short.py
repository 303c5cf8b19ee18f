"""Short per-kernel summary of a rocprofv3 kernel_stats.csv: name (trimmed), calls, avg us, %."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for x in rows[:n]:
    print(f"{x['Name'][:78]:80s} {int(x['Calls']):5d} {float(x['AverageNs']) / 1e3:9.1f}us {float(x['Percentage']):6.2f}%")
