"""Build libposecnn_hip.so in-tree for gfx950 (hipcc, no JIT cache)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libposecnn_hip.so")
SOURCES = ["capi.hip", "hough_compact.hip", "hough_vote.hip", "hough_peak.hip", "hough_emit.hip", "roi_pooling.hip", "average_distance.hip", "backprojecting.hip",
           "pose_head.hip"]
# -ffp-contract=off: the parity arithmetic rounds every float op separately
# (reference semantics restated by oracle/); MFMA kernels are unaffected.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wno-unused-result"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, "pcnn_common.h"), os.path.join(CSRC, "hough_common.h"),
                                                      os.path.join(HERE, "..", "include", "posecnn_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + FLAGS + ["-o", OUT + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
