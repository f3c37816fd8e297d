"""Per-launch HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes, plus
the VALUBusy of the voting kernels (scripts/gpu.sh pmc) -> profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM
section), so reads are doubled.  GEMM dispatches are told apart by their
fixed enqueue order inside a pose step (STEP_ORDER, pipeline.py).
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

# split-GEMM dispatches (k_gemm_x6 at the step's default precision, k_gemm_x3
# at precision 1) of one pose step in enqueue order (pipeline.py), over every
# tile / layout instantiation
STEP_ORDER = ["fc6_fwd", "fc7_fwd", "fc8_fwd", "fc8_dw", "fc8_dx", "fc7_dw", "fc7_dx", "fc6_dw", "fc6_dx"]
GEMM_FAMILIES = ("k_gemm_x6", "k_gemm_x3")


def gemm_roles(per, fam):
    """{role: [values]} from {kernel: [(dispatch_id, value)]}; roles by position in the step order."""
    seq = sorted(x for k, v in per.items() if k.startswith(fam) for x in v)
    out = defaultdict(list)
    for i, (_, val) in enumerate(seq):
        out[STEP_ORDER[i % len(STEP_ORDER)]].append(val)
    return out
HOUGH = ("k_label_hist", "k_label_place", "k_hough_vote", "k_hough_peak",
         "k_hough_emit", "k_hough_nms_cand", "k_hough_cand_data", "k_hough_nms_select")


def base(name):
    """Kernel name without its template arguments: the trace key of the vote
    is e.g. `k_hough_vote<4, 512>`, which must count as `k_hough_vote`."""
    return name.split("<", 1)[0]


def hough_keys(d):
    """The keys of d that are Hough-op kernels, matched on the base name (every
    template instantiation counts)."""
    return sorted(k for k in d if base(k) in HOUGH)


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0]


def load(path, counter):
    per = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        per[short(row["Kernel_Name"])].append((int(row["Dispatch_Id"]), float(row["Counter_Value"]) * 1024.0))
    for k in per:
        per[k].sort()
    return per


def summarize(fetch_csv, write_csv):
    f, w = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    out = {}
    for fam in GEMM_FAMILIES:
        fr_all, wr_all = gemm_roles(f, fam), gemm_roles(w, fam)
        for role, fr in fr_all.items():
            wr = wr_all.get(role, [])
            out[f"{fam}:{role}"] = {"read_bytes": 2 * sum(fr) / len(fr), "write_bytes": sum(wr) / max(len(wr), 1),
                                    "dispatches": len(fr)}
    for k in f:
        fv = [v for _, v in f[k]]
        wv = [v for _, v in w.get(k, [])]
        out[k] = {"read_bytes": 2 * sum(fv) / len(fv), "write_bytes": sum(wv) / max(len(wv), 1),
                  "dispatches": len(fv)}
    for v in out.values():
        v["traffic_bytes"] = v["read_bytes"] + v["write_bytes"]
    hk = hough_keys(out)
    if hk:
        out["hough_voting_gpu op"] = {"traffic_bytes": sum(out[k]["traffic_bytes"] for k in hk),
                                      "kernels": hk}
    return out


def valu_busy(path):
    """{kernel: mean rocprofv3 VALUBusy %} and the duration-weighted mean over
    the Hough op's kernels (derived metric, gfx94x formula on ROCm 7.2)."""
    if not os.path.exists(path):
        return None
    per, dur = defaultdict(list), defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != "VALUBusy":
            continue
        k = short(row["Kernel_Name"])
        per[k].append(float(row["Counter_Value"]))
        dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = {k: sum(v) / len(v) for k, v in per.items()}
    hk = hough_keys(out)
    if hk:
        tot = sum(sum(dur[k]) / len(dur[k]) for k in hk)
        out["hough_voting_gpu op"] = sum(out[k] * sum(dur[k]) / len(dur[k]) for k in hk) / tot
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    res = {"full": summarize(f"{root}/pmc_fetch/run_counter_collection.csv",
                             f"{root}/pmc_write/run_counter_collection.csv"),
           "vote_roi": summarize(f"{root}/pmc_fetch_vr/run_counter_collection.csv",
                                 f"{root}/pmc_write_vr/run_counter_collection.csv"),
           "note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 half-count), write = WRITE_SIZE; "
                   "valu_busy_pct = rocprofv3 VALUBusy (derived, gfx94x formula), duration-weighted over the op"}
    for wl, d in (("full", "pmc_valu"), ("vote_roi", "pmc_valu_vr")):
        vb = valu_busy(f"{root}/{d}/run_counter_collection.csv")
        for k, v in (vb or {}).items():
            if k in res[wl]:
                res[wl][k]["valu_busy_pct"] = round(v, 2)
    os.makedirs("profiles", exist_ok=True)
    json.dump(res, open("profiles/pmc_traffic.json", "w"), indent=1, sort_keys=True)
    for wl in ("full", "vote_roi"):
        for k, v in sorted(res[wl].items(), key=lambda kv: -kv[1]["traffic_bytes"])[:14]:
            vb = f"  VALUBusy {v['valu_busy_pct']:.1f} %" if "valu_busy_pct" in v else ""
            print(wl, k.ljust(40), f"{v['traffic_bytes'] / 1e6:10.2f} MB{vb}")


if __name__ == "__main__":
    main()
