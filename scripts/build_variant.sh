#!/bin/bash
# build_variant.sh NAME [-DFLAG ...]: the product library with extra defines,
# into scratch/NAME.so (gitignored, travels to the GPU box) for A/B runs
# selected with POSECNN_HIP_LIB.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p scratch
C=posecnn_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result "$@" \
  -o scratch/$name.so $C/capi.hip $C/hough_compact.hip $C/hough_vote.hip $C/hough_peak.hip $C/hough_emit.hip \
  $C/roi_pooling.hip $C/average_distance.hip $C/backprojecting.hip $C/pose_head.hip
