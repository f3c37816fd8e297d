"""Average rocprofv3 counter values per kernel: python scripts/sq_summary.py DIR [DIR ...] [--grep NAME]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--grep")]
pat = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--grep=")), "")
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, c in agg.items():
            print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
