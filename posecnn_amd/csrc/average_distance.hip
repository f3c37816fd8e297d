// ADD / ADD-S pose loss for PoseCNN on MI355X (gfx950).
//
// Replaces AveragedistanceForwardLaucher / AveragedistanceBackwardLaucher
// (lib/average_distance_loss/average_distance_loss_op_gpu.cu.cc:34-377).
//
// The reference runs one thread per (row, point), re-deriving the row's six
// 3x3 matrices per point into a (R, P, 54) global scratch and the per-point
// gradient into a (R, P, 4C) scratch (~0.64 GB at R = 432), then sums both
// sequentially per row and reduces the row losses with thrust + a host copy.
// Here a workgroup owns (row, chunk of 256 points): the matrices are computed
// once in registers, symmetric classes stage the GT-rotated model points in
// LDS for the O(P) nearest-point search, and the per-point loss and the four
// gradient terms are reduced in a fixed tree -> (R, chunks, 5) partials.
// A single workgroup then folds the partials per row and the rows into the
// scalar loss, both in fixed order (deterministic; the reference's sequential
// sums are reproduced to fp32 rounding, tolerance 1e-4 relative).
#include "pcnn_common.h"
#include <cfloat>

namespace {

constexpr int kAddThreads = 256;
constexpr int kMaxPointsLds = 4096;

__device__ __forceinline__ int rows_of(const int32_t* dev, int cap) {
  if (!dev) return cap;
  int r = *dev;
  return r < cap ? r : cap;
}

// cu.cc:63-71 (unnormalised quaternion -> rotation)
__device__ __forceinline__ void quat2rot(float s, float u, float v, float w, float* r) {
  r[0] = s * s + u * u - v * v - w * w;
  r[1] = 2 * (u * v - s * w);
  r[2] = 2 * (u * w + s * v);
  r[3] = 2 * (u * v + s * w);
  r[4] = s * s - u * u + v * v - w * w;
  r[5] = 2 * (v * w - s * u);
  r[6] = 2 * (u * w - s * v);
  r[7] = 2 * (v * w + s * u);
  r[8] = s * s - u * u - v * v + w * w;
}

__global__ void __launch_bounds__(kAddThreads) k_add_rows(const float* __restrict__ pred,
                                                           const float* __restrict__ target,
                                                           const float* __restrict__ weight,
                                                           const float* __restrict__ points,
                                                           const float* __restrict__ symmetry, int R_cap,
                                                           const int32_t* __restrict__ num_rois_dev, int C, int P,
                                                           float margin, int norm_rows,
                                                           const int32_t* __restrict__ norm_rows_dev, int nchunk,
                                                           float* __restrict__ partial) {
  __shared__ float gpts[kMaxPointsLds * 3];
  __shared__ float red[kAddThreads / 64][5];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int R = rows_of(num_rois_dev, R_cap);
  if (n >= R) return;
  const int PC = 4 * C;
  int cls = -1;
  for (int i = 0; i < C; i++)  // first class with weight > 0 (cu.cc:47-52)
    if (weight[(size_t)n * PC + 4 * i] > 0) { cls = i; break; }
  float* out = partial + ((size_t)n * nchunk + chunk) * 5;
  if (cls < 0) {
    if (threadIdx.x < 5) out[threadIdx.x] = 0.f;
    return;
  }
  const float* tq = target + (size_t)n * PC + 4 * cls;
  const float* pq = pred + (size_t)n * PC + 4 * cls;
  float Rg[9], Rp[9];
  quat2rot(tq[0], tq[1], tq[2], tq[3], Rg);
  const float s = pq[0], u = pq[1], v = pq[2], w = pq[3];
  quat2rot(s, u, v, w, Rp);
  // derivative matrices of Rp w.r.t. (s, u, v, w) (cu.cc:97-139)
  const float d0[9] = {2 * s, -2 * w, 2 * v, 2 * w, 2 * s, -2 * u, -2 * v, 2 * u, 2 * s};
  const float d1[9] = {2 * u, 2 * v, 2 * w, 2 * v, -2 * u, -2 * s, 2 * w, 2 * s, -2 * u};
  const float d2[9] = {-2 * v, 2 * u, 2 * s, 2 * u, 2 * v, 2 * w, -2 * s, 2 * w, -2 * v};
  const float d3[9] = {-2 * w, -2 * s, 2 * u, 2 * s, -2 * w, 2 * v, 2 * u, 2 * v, 2 * w};
  const float* pts = points + (size_t)cls * P * 3;
  const bool sym = symmetry[cls] > 0;
  if (sym) {
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
      const float X0 = pts[i * 3 + 0], X1 = pts[i * 3 + 1], X2 = pts[i * 3 + 2];
      gpts[i * 3 + 0] = Rg[0] * X0 + Rg[1] * X1 + Rg[2] * X2;
      gpts[i * 3 + 1] = Rg[3] * X0 + Rg[4] * X1 + Rg[5] * X2;
      gpts[i * 3 + 2] = Rg[6] * X0 + Rg[7] * X1 + Rg[8] * X2;
    }
    __syncthreads();
  }
  const int Rn = norm_rows_dev ? *norm_rows_dev : (norm_rows > 0 ? norm_rows : R);
  const float bn = (float)(Rn * P);
  const double ln = 2.0 * (double)Rn * (double)P;
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  const int p = chunk * blockDim.x + threadIdx.x;
  if (p < P) {
    const float X0 = pts[p * 3 + 0], X1 = pts[p * 3 + 1], X2 = pts[p * 3 + 2];
    const float x1 = Rp[0] * X0 + Rp[1] * X1 + Rp[2] * X2;
    const float y1 = Rp[3] * X0 + Rp[4] * X1 + Rp[5] * X2;
    const float z1 = Rp[6] * X0 + Rp[7] * X1 + Rp[8] * X2;
    float x2, y2, z2;
    if (sym) {  // closest GT-rotated point, first minimum (cu.cc:150-168)
      float dmin = FLT_MAX;
      int imin = p;
      for (int i = 0; i < P; i++) {
        const float ax = gpts[i * 3 + 0], ay = gpts[i * 3 + 1], az = gpts[i * 3 + 2];
        const float dist = (x1 - ax) * (x1 - ax) + (y1 - ay) * (y1 - ay) + (z1 - az) * (z1 - az);
        if (dist < dmin) { dmin = dist; imin = i; }
      }
      x2 = gpts[imin * 3 + 0];
      y2 = gpts[imin * 3 + 1];
      z2 = gpts[imin * 3 + 2];
    } else {
      x2 = Rg[0] * X0 + Rg[1] * X1 + Rg[2] * X2;
      y2 = Rg[3] * X0 + Rg[4] * X1 + Rg[5] * X2;
      z2 = Rg[6] * X0 + Rg[7] * X1 + Rg[8] * X2;
    }
    const float dist = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2);
    if (!(dist < margin)) {  // cu.cc:178-179
      acc[0] = (float)((double)(dist - margin) / ln);
      const float X[3] = {X0, X1, X2};
      const float df[3] = {x1 - x2, y1 - y2, z1 - z2};
#pragma unroll
      for (int j = 0; j < 3; j++)
#pragma unroll
        for (int k = 0; k < 3; k++) {  // cu.cc:183-203, same operation order
          acc[1] += df[j] * X[k] * d0[j * 3 + k] / bn;
          acc[2] += df[j] * X[k] * d1[j * 3 + k] / bn;
          acc[3] += df[j] * X[k] * d2[j * 3 + k] / bn;
          acc[4] += df[j] * X[k] * d3[j * 3 + k] / bn;
        }
    }
  }
#pragma unroll
  for (int q = 0; q < 5; q++) acc[q] = pcnn::wave_sum(acc[q]);
  const int wv = threadIdx.x >> 6;
  if (pcnn::lane_id() == 0)
    for (int q = 0; q < 5; q++) red[wv][q] = acc[q];
  __syncthreads();
  if (threadIdx.x < 5) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i][threadIdx.x];
    out[threadIdx.x] = t;
  }
}

// One workgroup: per-row fold of the chunk partials, bottom_diff rows, loss.
__global__ void __launch_bounds__(1024) k_add_finish(const float* __restrict__ weight, int R_cap,
                                                      const int32_t* __restrict__ num_rois_dev, int C, int nchunk,
                                                      const float* __restrict__ partial, float* __restrict__ loss,
                                                      float* __restrict__ bottom_diff) {
  __shared__ float red[16];
  const int R = rows_of(num_rois_dev, R_cap);
  const int PC = 4 * C;
  float my = 0.f;
  for (int n = threadIdx.x; n < R; n += blockDim.x) {
    int cls = -1;
    for (int i = 0; i < C; i++)
      if (weight[(size_t)n * PC + 4 * i] > 0) { cls = i; break; }
    float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nchunk; k++)
      for (int q = 0; q < 5; q++) s[q] += partial[((size_t)n * nchunk + k) * 5 + q];
    float* bd = bottom_diff + (size_t)n * PC;
    for (int t = 0; t < PC; t++) bd[t] = 0.f;
    if (cls >= 0)
      for (int q = 0; q < 4; q++) bd[4 * cls + q] = s[q + 1];
    my += cls >= 0 ? s[0] : 0.f;
  }
  my = pcnn::wave_sum(my);
  if (pcnn::lane_id() == 0) red[threadIdx.x >> 6] = my;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
    loss[0] = t;
  }
}

__global__ void k_add_bwd(const float* __restrict__ top_diff, const float* __restrict__ bottom_diff, int n,
                          float* __restrict__ out) {
  const float g = top_diff[0];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = g * bottom_diff[i];
}

__global__ void k_add_bwd_rows(const float* __restrict__ top_diff, const float* __restrict__ bottom_diff,
                               const int32_t* __restrict__ num_rois_dev, int R_cap, int row_len,
                               float* __restrict__ out) {
  const float g = top_diff[0];
  const int n = rows_of(num_rois_dev, R_cap) * row_len;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = g * bottom_diff[i];
}

}  // namespace

extern "C" size_t pcnn_add_loss_workspace_size(int R_cap, int C, int P) {
  (void)C;
  const int nchunk = (P + kAddThreads - 1) / kAddThreads;
  return pcnn::align_up((size_t)(R_cap > 0 ? R_cap : 1) * nchunk * 5 * sizeof(float), 256) + 256;
}

extern "C" int pcnn_add_loss_fwd(const float* pred, const float* target, const float* weight, const float* points,
                                 const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P,
                                 float margin, int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss,
                                 float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(pred && target && weight && points && symmetry && loss && bottom_diff && workspace);
  PCNN_REQUIRE(R_cap > 0 && C > 0 && P > 0 && P <= kMaxPointsLds);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = (P + kAddThreads - 1) / kAddThreads;
  float* partial = (float*)workspace;
  hipLaunchKernelGGL(k_add_rows, dim3(nchunk, R_cap), dim3(kAddThreads), 0, st, pred, target, weight, points,
                     symmetry, R_cap, num_rois_dev, C, P, margin, loss_norm_rows, loss_norm_rows_dev, nchunk,
                     partial);
  hipLaunchKernelGGL(k_add_finish, dim3(1), dim3(1024), 0, st, weight, R_cap, num_rois_dev, C, nchunk, partial, loss,
                     bottom_diff);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_add_loss_bwd(const float* top_diff, const float* bottom_diff, int n,
                                 const int32_t* num_rois_dev, int row_len, float* out, void* stream) {
  PCNN_REQUIRE(top_diff && bottom_diff && out && n >= 0);
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return PCNN_OK;
  const int blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  if (num_rois_dev) {
    PCNN_REQUIRE(row_len > 0);
    hipLaunchKernelGGL(k_add_bwd_rows, dim3(blocks), dim3(256), 0, st, top_diff, bottom_diff, num_rois_dev,
                       n / row_len, row_len, out);
  } else {
    hipLaunchKernelGGL(k_add_bwd, dim3(blocks), dim3(256), 0, st, top_diff, bottom_diff, n, out);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
