"""Per-role average durations of the GEMM dispatches in a rocprofv3
kernel_trace.csv (roles by fixed launch order per pose step, as
scripts/pmc_traffic.py), to check bench.py's HIP-event roofline timing."""
import csv
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_traffic import GEMM_FAMILIES, STEP_ORDER, gemm_roles  # noqa: E402

per = defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", row["Kernel_Name"])
    if m:
        per[m.group(1)].append((int(row["Dispatch_Id"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3))
for fam in GEMM_FAMILIES:
    roles = gemm_roles(per, fam)
    for role in STEP_ORDER:
        x = roles.get(role, [])
        if x:
            print(f"{fam}:{role:8s} n={len(x):4d} avg={sum(x) / len(x):8.1f} us")
