"""Per-role DRAM vs fabric reads of the step's GEMMs and Hough / RoI kernels
from a rocprofv3 --pmc pass of TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum and
TCC_EA0_RDREQ_DRAM_sum (scripts/gpu.sh dram): EA read requests are the L2's
misses, served by the 256 MB MALL (Infinity Cache) or by HBM; the _DRAM ones
reached HBM.  Bytes = 64 per request (32 for the 32-B ones), as the guide's
FETCH_SIZE expression counts them.
    python scripts/dram_split.py DIR"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_traffic import GEMM_FAMILIES, gemm_roles, short  # noqa: E402

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(list))
for row in csv.DictReader(open(f)):
    per[row["Counter_Name"]][short(row["Kernel_Name"])].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
out = {}
for fam in GEMM_FAMILIES:
    roles = {c: gemm_roles(per[c], fam) for c in per}
    for role in roles.get("TCC_EA0_RDREQ_sum", {}):
        v = {c: sum(roles[c][role]) / len(roles[c][role]) for c in roles if roles[c].get(role)}
        rd, r32, dram = v.get("TCC_EA0_RDREQ_sum", 0), v.get("TCC_EA0_RDREQ_32B_sum", 0), v.get("TCC_EA0_RDREQ_DRAM_sum", 0)
        out[f"{fam}:{role}"] = {"ea_read_MB": round(((rd - r32) * 64 + r32 * 32) / 1e6, 1),
                                "dram_read_requests_frac": round(dram / rd, 3) if rd else None}
print(json.dumps(out, indent=1))
