"""Print the kernel timeline of one pose step from a rocprofv3 kernel_trace.csv
(start / end relative to the step's first kernel, duration, name).
    python scripts/timeline.py DIR/run_kernel_trace.csv [step_from_end]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ev = []
for r in rows:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:40]))
ev.sort()
idx = [i for i, e in enumerate(ev) if e[2] == "k_label_hist"]
a, b = idx[-back - 1], idx[-back]
t0 = ev[a][0]
for s, e, n in ev[a:b]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n[:60]}")
print(f"step span {(ev[b][0] - t0) / 1e3:.1f} us")
