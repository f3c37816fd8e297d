// Label producers in front of the Hough vote.
//
//  argmax_2d  label_2d = argmax over the class axis of prob_normalized
//             (lib/networks/network.py:433-434, fed by vgg16_convs.py:144-146):
//             a pure HBM stream of B*H*W*C*4 bytes in, B*H*W*4 out.  The
//             fused form inside the Hough op is k_label_hist_prob
//             (hough_compact.hip); this stand-alone kernel serves callers that
//             only need label_2d.
//  Hardlabel  one-hot GT label weights (lib/hard_label_layer/
//             hard_label_op_gpu.cu.cc:17-29, grad :56-64), written as a single
//             coalesced stream of the (B,H,W,C) output.
//  vertex_pred, class-compact: the 1x1 conv 128 -> 3C
//             + bias of vgg16_convs.py:152-163 evaluated only at the 3
//             channels of each pixel's label class, written as (B,H,W,3):
//             12 B/px instead of the 264 B/px (C = 22) map the Hough op
//             reads ~2 % of.
#include "hough_common.h"

namespace {

using namespace pcnn_hough;

constexpr int kArgThreads = 256;

__global__ void __launch_bounds__(kArgThreads) k_argmax_2d(const float* __restrict__ prob, int HW, int C,
                                                           int32_t* __restrict__ label) {
  extern __shared__ __attribute__((aligned(16))) float stage_all[];
  const int b = blockIdx.y;
  const float* img = prob + (size_t)b * HW * C;
  float* stage = stage_all + (threadIdx.x >> 6) * 64 * (C <= kArgmaxStagedMaxC ? C : 0);
  const int p0 = blockIdx.x * kArgThreads + (threadIdx.x & ~63);
  const int l = wave_argmax_rows(img, p0, HW, C, stage);
  const int p = p0 + pcnn::lane_id();
  if (p < HW) label[(size_t)b * HW + p] = l;
}

// One thread per 4 consecutive output elements (float4 store) of the
// (pixels x classes) output: the reference's per-pixel zero-fill plus one-hot
// store (cu.cc:21-27) as one coalesced write stream.  A gt label outside
// [-1, C) indexes past the pixel's row in the reference (undefined); here it
// yields an all-zero row.
__device__ __forceinline__ float hard_label_at(const float* __restrict__ prob, const int32_t* __restrict__ gt,
                                               int pix, int c, int C, float threshold) {
  const int g = gt[pix];
  return (c == g && g >= 0 && g < C && (g > 0 || prob[(size_t)pix * C + g] < threshold)) ? 1.f : 0.f;  // cu.cc:25-26
}

__global__ void __launch_bounds__(256) k_hard_label(const float* __restrict__ prob, const int32_t* __restrict__ gt,
                                                    int n_pix, int C, float threshold, float* __restrict__ top) {
  const int total = n_pix * C;
  const int n4 = total / 4;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
    int pix = (4 * q) / C;
    int c = 4 * q - pix * C;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j] = hard_label_at(prob, gt, pix, c, C, threshold);
      if (++c == C) { c = 0; pix++; }
    }
    ((float4*)top)[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
  if (blockIdx.x == 0 && (int)threadIdx.x < total - 4 * n4) {  // ragged tail (< 4 elements)
    const int i = 4 * n4 + threadIdx.x;
    top[i] = hard_label_at(prob, gt, i / C, i % C, C, threshold);
  }
}

// One thread per pixel over a persistent grid; the (K, 3C) weights sit in
// LDS.  out[j] = (sum over k in order of feat[k] * w[k][3l + j]) + bias[3l + j]
// (conv2d then bias_add, network.py:168-185), every op rounded separately.
// A label outside [0, C) writes zeros (the vote never reads such pixels).
constexpr int kVpThreads = 256;
__global__ void __launch_bounds__(kVpThreads) k_vertex_pred_compact(const float* __restrict__ feat,
                                                                    const float* __restrict__ w,
                                                                    const float* __restrict__ bias,
                                                                    const int32_t* __restrict__ label, long n_pix,
                                                                    int K, int C, float* __restrict__ out) {
  extern __shared__ float wl[];  // [K][3C]
  const int NC3 = 3 * C;
  for (int i = threadIdx.x; i < K * NC3; i += blockDim.x) wl[i] = w[i];
  __syncthreads();
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < n_pix; p += (long)gridDim.x * blockDim.x) {
    const int l = label[p];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    if (l >= 0 && l < C) {
      const float4* x4 = (const float4*)(feat + p * K);
      const float* wc = wl + 3 * l;
      for (int k4 = 0; k4 < K / 4; k4++) {
        const float4 x = x4[k4];
        const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const float* wr = wc + (4 * k4 + e) * NC3;
          a0 = a0 + xv[e] * wr[0];
          a1 = a1 + xv[e] * wr[1];
          a2 = a2 + xv[e] * wr[2];
        }
      }
      a0 = a0 + bias[3 * l + 0];
      a1 = a1 + bias[3 * l + 1];
      a2 = a2 + bias[3 * l + 2];
    }
    out[p * 3 + 0] = a0;
    out[p * 3 + 1] = a1;
    out[p * 3 + 2] = a2;
  }
}

inline size_t argmax_lds(int C) { return C <= kArgmaxStagedMaxC ? (size_t)(kArgThreads / 64) * 64 * C * 4 : 0; }

}  // namespace

extern "C" int pcnn_argmax_2d(const float* prob, int B, int H, int W, int C, int32_t* label, void* stream) {
  PCNN_REQUIRE(prob && label && B > 0 && H > 0 && W > 0 && C > 0);
  PCNN_REQUIRE((long)H * W * C < (1l << 31));
  const int HW = H * W;
  hipLaunchKernelGGL(k_argmax_2d, dim3((HW + kArgThreads - 1) / kArgThreads, B), dim3(kArgThreads), argmax_lds(C),
                     (hipStream_t)stream, prob, HW, C, label);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hard_label_fwd(const float* prob, const int32_t* gt, int B, int H, int W, int C, float threshold,
                                   float* top, void* stream) {
  PCNN_REQUIRE(prob && gt && top && B > 0 && H > 0 && W > 0 && C > 0);
  PCNN_REQUIRE(threshold > 0.f);  // hard_label_op.cc:50-52 (attr check)
  PCNN_REQUIRE((long)B * H * W * C < (1l << 31));
  PCNN_REQUIRE((((uintptr_t)top) & 15) == 0);  // float4 stores
  const int n_pix = B * H * W;
  const long n4 = (long)n_pix * C / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_hard_label, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, prob, gt, n_pix, C,
                     threshold, top);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hard_label_bwd(float* grad_prob, float* grad_gt, int B, int H, int W, int C, void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0);
  hipStream_t st = (hipStream_t)stream;
  const size_t n_pix = (size_t)B * H * W;
  if (grad_prob && hipMemsetAsync(grad_prob, 0, n_pix * C * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
  if (grad_gt && hipMemsetAsync(grad_gt, 0, n_pix * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_vertex_pred_compact(const float* feat, const float* weights, const float* bias,
                                        const int32_t* label, int B, int H, int W, int K, int C, float* vertex3,
                                        void* stream) {
  PCNN_REQUIRE(feat && weights && bias && label && vertex3 && B > 0 && H > 0 && W > 0 && C > 0);
  PCNN_REQUIRE(K > 0 && K % 4 == 0 && (((uintptr_t)feat) & 15) == 0);
  const size_t lds = (size_t)K * 3 * C * sizeof(float);
  PCNN_REQUIRE(lds <= 64 * 1024);
  const long n_pix = (long)B * H * W;
  long blocks = (n_pix + kVpThreads - 1) / kVpThreads;
  if (blocks > 256 * 4) blocks = 256 * 4;  // persistent: the weights are staged once per workgroup
  hipLaunchKernelGGL(k_vertex_pred_compact, dim3((unsigned)blocks), dim3(kVpThreads), lds, (hipStream_t)stream, feat,
                     weights, bias, label, n_pix, K, C, vertex3);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
