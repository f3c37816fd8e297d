// The pose head's backward for one RoI row (tanh * poses_weight ->
// tf.nn.l2_normalize, vgg16_convs.py:193-197, network.py:440-445): one wave
// per row, D <= 256 columns at lane + 64 k.  Shared by k_head_bwd
// (pose_head.hip, d_pred read from memory) and the ADD loss's fused tail
// (average_distance.hip, d_pred straight from the row's finished sums), so
// both give the same bits.
#pragma once
#include "pcnn_common.h"

namespace pcnn_head {

// dp[k] = d loss / d pred at column lane + 64 k (already scaled by the ADD
// gradient op's top_diff[0]; 0 past D)
__device__ __forceinline__ void head_bwd_row(const float (&dp)[4], const float* __restrict__ t_in,
                                             const float* __restrict__ pw, const float* __restrict__ pred, int row,
                                             int D, int lane, float* __restrict__ dy8) {
  float ss = 0.f, dot = 0.f;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    if (c < D) {
      const float mv = t_in[(size_t)row * D + c] * pw[(size_t)row * D + c];
      ss += mv * mv;
      dot += pred[(size_t)row * D + c] * dp[k];
    }
  }
  ss = pcnn::wave_sum(ss);
  dot = pcnn::wave_sum(dot);
  const bool clamp = !(ss > 1e-12f);
  const float inv = 1.f / sqrtf(fmaxf(ss, 1e-12f));
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    if (c < D) {
      const size_t o = (size_t)row * D + c;
      // d/dm of m * rsqrt(max(sum m^2, eps))
      const float dm = clamp ? dp[k] * inv : (dp[k] - pred[o] * dot) * inv;
      const float dt = dm * pw[o];
      const float t = t_in[o];
      dy8[o] = dt * (1.f - t * t);
    }
  }
}

}  // namespace pcnn_head
