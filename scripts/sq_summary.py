"""Per-kernel averages of SQ counters from scripts/gpu_sq.sh output."""
import csv
import re
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for d in ("sq1", "sq2"):
    for row in csv.DictReader(open(f"gpurun_out/{d}/run_counter_collection.csv")):
        m = re.search(r"(k_\w+(?:<[^>]*>)?)", row["Kernel_Name"])
        if not m:
            continue
        k = m.group(1)
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k][row["Counter_Name"]] += 1
want = sys.argv[1:] or None
for k in sorted(agg):
    if want and not any(w in k for w in want):
        continue
    a = {c: agg[k][c] / cnt[k][c] for c in agg[k]}
    wc = a.get("SQ_WAVE_CYCLES", 1) or 1
    gui = a.get("GRBM_GUI_ACTIVE", 0) / 8
    print(f"{k:45s} gui_cyc={gui:9.0f} waves={a.get('SQ_WAVES', 0):7.0f} wait={a.get('SQ_WAIT_ANY', 0) / wc:5.2f} "
          f"stall={a.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} active={a.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} "
          f"valu={a.get('SQ_INSTS_VALU', 0):10.0f} lds={a.get('SQ_INSTS_LDS', 0):9.0f} vmem={a.get('SQ_INSTS_VMEM', 0):8.0f} "
          f"salu={a.get('SQ_INSTS_SALU', 0):8.0f} ldsconf={a.get('SQ_LDS_BANK_CONFLICT', 0) / max(a.get('SQ_LDS_IDX_ACTIVE', 1), 1):4.2f} "
          f"mfma%={a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(gui * 1024, 1) * 100:5.1f}")
