"""Back-projection HBM traffic by rocprofv3 counters beside the algorithmic
bytes of scripts/bp_bench.py (VERDICT r04 "what's weak" #9: the backward's
algorithmic rate counts one gradient-row read per in-grid pixel, which is not
HBM traffic where pixels share a voxel).

usage: python scripts/bp_pmc.py OUT_DIR BENCH_JSON
OUT_DIR holds bp_{scene}_{fetch,write}/run_counter_collection.csv from
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes over
`bp_bench.py --scene {scene}` (scripts/gpu.sh bppmc).  Reads are 2 x
FETCH_SIZE (gfx950 counts half the bytes of wide coalesced reads,
MI355X_MICROARCH.md HBM section).  Prints BENCH_JSON with, per scene and
direction, pmc_bytes (per launch), pmc_TBps (over the bench's HIP-event
time) and algorithmic_over_pmc."""
import csv
import json
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    d = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter and "k_bp_" in row["Kernel_Name"]:
            name = re.search(r"(k_bp_\w+(?:<[^>]*>)?)", row["Kernel_Name"]).group(1)
            d[name].append(float(row["Counter_Value"]) * 1024.0)
    return d


def main():
    out_dir, bench = sys.argv[1], json.load(open(sys.argv[2]))
    for scene in ("scene", "objects"):
        if scene not in bench:
            continue
        f = per_kernel(f"{out_dir}/bp_{scene}_fetch/run_counter_collection.csv", "FETCH_SIZE")
        w = per_kernel(f"{out_dir}/bp_{scene}_write/run_counter_collection.csv", "WRITE_SIZE")
        r = bench[scene]
        for direction, pred in (("fwd", lambda k: "bwd" not in k), ("bwd", lambda k: "bwd" in k)):
            ks = [k for k in f if pred(k)]
            if not ks:
                continue
            k = ks[0]
            byt = 2 * sum(f[k]) / len(f[k]) + sum(w.get(k, [0.0])) / max(len(w.get(k, [])), 1)
            r[f"{direction}_pmc_kernel"] = k
            r[f"{direction}_pmc_bytes"] = round(byt)
            r[f"{direction}_pmc_TBps"] = round(byt / r[f"{direction}_us"] / 1e6, 3)
            r[f"{direction}_algorithmic_over_pmc"] = round(r[f"{direction}_algorithmic_bytes"] / byt, 3)
    bench["pmc_note"] = ("pmc_bytes = 2 x FETCH_SIZE + WRITE_SIZE per launch (rocprofv3, separate passes); "
                         "pmc_TBps = pmc_bytes / the bench's HIP-event time per launch")
    print(json.dumps(bench))


if __name__ == "__main__":
    main()
