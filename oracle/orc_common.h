// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference PoseCNN hot-path ops (mrlooi/PoseCNN,
// lib/hough_voting_gpu_layer, lib/roi_pooling_layer, lib/average_distance_loss,
// lib/backprojecting_layer, lib/hough_voting_layer).  It is the *checker* for
// the HIP product path and the CPU baseline for bench.py; nothing in
// posecnn_amd/ may include, link or call it.
//
// Parity status: UNPINNED.  The reference ships no golden vectors, no
// known-answer tests and cannot be compiled here (TensorFlow headers, nvcc,
// thrust, Eigen, OpenCV, NLopt are all absent).  This
// restatement follows the reference source line by line (cited per function),
// is compiled with -ffp-contract=off (every float op rounds separately), and is
// pinned by hand-derived known-answer tests in tests/test_oracle_kat.py.
//
// Written independently of posecnn_amd/csrc: it shares no source with the
// product.
#pragma once
#include <cstdint>
#include <cmath>
#include <cfloat>
#include <climits>

#define ORC_API extern "C" __attribute__((visibility("default")))

namespace orc {

// exp() of the vertex-map depth channel.  The reference evaluates CUDA
// libdevice expf (hough_voting_gpu_op.cu.cc:280), which is not reproducible
// off-GPU; this restatement pins d = round_to_float(exp((double)z)).
inline float exp_depth(float z) { return (float)std::exp((double)z); }

// float -> int conversion with GPU semantics (NaN -> 0, saturating), used where
// the reference converts a possibly non-finite float to int (backproject
// round(), roi coordinates).  C++ leaves these cases undefined.
inline int f2i_sat(float f) {
  if (std::isnan(f)) return 0;
  if (f >= 2147483648.0f) return INT_MAX;
  if (f <= -2147483648.0f) return INT_MIN;
  return (int)f;
}

}  // namespace orc
