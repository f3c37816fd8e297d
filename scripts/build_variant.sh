#!/bin/bash
# build_variant.sh NAME [-DFLAG ...]: the product library with extra defines,
# into scratch/NAME.so (gitignored, travels to the GPU box) for A/B runs
# selected with POSECNN_HIP_LIB.  REV=<git rev> builds that revision's
# sources instead of the working tree (e.g. REV=HEAD for a before/after A/B).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p scratch/$name.obj
C=posecnn_amd/csrc
if [ -n "$REV" ]; then
  src=scratch/$name.src; rm -rf $src; mkdir -p $src
  git archive "$REV" posecnn_amd/csrc include | tar -x -C $src
  C=$src/posecnn_amd/csrc
fi
pids=""
for f in $(python3 -c "import sys; sys.path.insert(0, '.'); from posecnn_amd.build import SOURCES; print(' '.join(s[:-4] for s in SOURCES))"); do
  [ -f $C/$f.hip ] || continue  # a source the built revision does not have
  extra=""; { [ $f = pose_head ] || [ $f = gemm_x6 ] || [ $f = gemm_tp ]; } && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-result $extra "$@" \
    -c $C/$f.hip -o scratch/$name.obj/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scratch/$name.so scratch/$name.obj/*.o
rm -rf scratch/$name.obj scratch/$name.src
