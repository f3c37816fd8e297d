"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg us, share."""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")))
tot = sum(float(x["TotalDurationNs"]) for x in r)
for x in r[:int(sys.argv[2]) if len(sys.argv) > 2 else 26]:
    print(x["Name"][:70].ljust(72), x["Calls"].rjust(5), f"{float(x['AverageNs']) / 1e3:9.1f}",
          f"{float(x['TotalDurationNs']) / tot * 100:6.1f}")
