"""Print the rocprofv3 kernel_stats.csv under a directory: name, calls, avg us, % of total."""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} {float(r['Percentage']):6.1f}")
