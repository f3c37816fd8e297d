// Class-aware greedy box NMS + pose combination on the device (SURVEY §8(f)
// rank 1): the inference consumer of the Hough op's RoI rows.
//
// Replaces, on the device, lib/utils/nms.py:3-32 (numpy NMS over the
// `rois` the Hough op returns) and the pose combination of
// lib/fcn/test.py:197-211:
//   keep = nms(rois, 0.5); rois = rois[keep]; poses = poses_init[keep];
//   poses[i, :4] = poses_pred[keep[i], 4*cls : 4*cls + 4] for cls >= 0.
//
// One workgroup: (1) rows sorted by score descending (64-bit keys, bitonic in
// LDS; numpy's argsort()[::-1] leaves the order of equal scores unspecified
// — here ties go to the lower row index, a canonical legal order); (2) the
// pairwise suppression bits of the sorted rows (ovr > thresh and same class,
// in the reference's float32 operation order) into an upper-triangular
// bitmask in LDS; (3) one wave walks the sorted rows, keeping a row when no
// kept row has suppressed it and OR-ing its mask row into the removed set held
// across the lanes (64 rows per lane word); (4) the kept rows are gathered.
#include "pcnn_common.h"

namespace {

constexpr int kNmsThreads = 1024;
constexpr int kNmsMaxRows = 1152;  // MAX_ROI * 9, the Hough op's row capacity (hough_voting_gpu_op.cc:94)
constexpr int kNmsWords = kNmsMaxRows / 64;
constexpr int kNmsTri = 64 * kNmsWords * (kNmsWords + 1) / 2;  // upper-triangular mask words

// first mask word of sorted row k: rows of 64-row block q keep words q .. nw-1
__device__ __forceinline__ int tri_off(int k, int nw) {
  const int q = k >> 6;
  return 64 * (q * nw - q * (q - 1) / 2) + (k & 63) * (nw - q);
}

__device__ __forceinline__ int rows_of(const int32_t* dev, int cap) {
  if (!dev) return cap;
  const int r = *dev;
  return r < 0 ? 0 : (r < cap ? r : cap);
}

// ascending key <=> score descending, then row ascending; NaN first (numpy
// sorts NaN last, reversed -> first), -0 == +0
__device__ __forceinline__ unsigned long long sort_key(float s, int row) {
  unsigned u = __float_as_uint(s == 0.f ? 0.f : s);
  unsigned mono = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving
  if (s != s) mono = 0xFFFFFFFFu;
  return ((unsigned long long)(~mono) << 32) | (unsigned)row;
}

__global__ void __launch_bounds__(kNmsThreads) k_box_nms(const float* __restrict__ rois, int R_cap, int stride,
                                                          const int32_t* __restrict__ num_rois_dev, float thresh,
                                                          int32_t* __restrict__ keep, int32_t* __restrict__ num_keep,
                                                          const float* __restrict__ poses_init,
                                                          const float* __restrict__ poses_pred, int pred_dim,
                                                          float* __restrict__ rois_out,
                                                          float* __restrict__ poses_out) {
  __shared__ unsigned long long key[kNmsMaxRows + 1024];  // padded to a power of two for the sort
  __shared__ unsigned long long mask[kNmsTri];
  __shared__ int s_nkeep;
  const int R = rows_of(num_rois_dev, R_cap);
  int n2 = 1;
  while (n2 < R) n2 <<= 1;  // <= 2048
  for (int i = threadIdx.x; i < n2; i += blockDim.x)
    key[i] = i < R ? sort_key(rois[(size_t)i * stride + 6], i) : ~0ull;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int st = size >> 1; st > 0; st >>= 1) {
      for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const int j = i ^ st;
        if (j > i) {
          const bool up = (i & size) == 0;
          const unsigned long long a = key[i], b = key[j];
          if ((a > b) == up) { key[i] = b; key[j] = a; }
        }
      }
      __syncthreads();
    }
  // (2) suppression bits of sorted row k over sorted rows l > k (nms.py:17-28)
  const int nw = (R + 63) / 64;
  const float th = thresh;
  for (int t = threadIdx.x; t < R * nw; t += blockDim.x) {
    const int k = t / nw, w = t % nw;
    if (w < (k >> 6)) continue;  // below the diagonal block: never read
    const int i = (int)(key[k] & 0xFFFFFFFFu);
    const float* ri = rois + (size_t)i * stride;
    const float ci = ri[1], x1 = ri[2], y1 = ri[3], x2 = ri[4], y2 = ri[5];
    const float ai = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);  // areas (nms.py:11)
    unsigned long long bits = 0ull;
    for (int b = 0; b < 64; b++) {
      const int l = w * 64 + b;
      if (l <= k || l >= R) continue;
      const int j = (int)(key[l] & 0xFFFFFFFFu);
      const float* rj = rois + (size_t)j * stride;
      const float aj = (rj[4] - rj[2] + 1.f) * (rj[5] - rj[3] + 1.f);
      const float xx1 = fmaxf(x1, rj[2]), yy1 = fmaxf(y1, rj[3]);
      const float xx2 = fminf(x2, rj[4]), yy2 = fminf(y2, rj[5]);
      const float ww = fmaxf(0.f, xx2 - xx1 + 1.f), hh = fmaxf(0.f, yy2 - yy1 + 1.f);
      const float inter = ww * hh;
      const float ovr = inter / (ai + aj - inter);  // nms.py:17-25
      if (ovr > th && rj[1] == ci) bits |= 1ull << b;  // nms.py:27
    }
    mask[tri_off(k, nw) + (w - (k >> 6))] = bits;
  }
  __syncthreads();
  // (3) greedy walk (nms.py:15-30): lane w holds removed-set word w as two
  // 32-bit halves (readlane with a uniform lane index)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned lo = 0u, hi = 0u;
    int nk = 0;
    for (int k = 0; k < R; k++) {
      const int b = k & 63;
      const unsigned v = b < 32 ? __builtin_amdgcn_readlane(lo, k >> 6) : __builtin_amdgcn_readlane(hi, k >> 6);
      if ((v >> (b & 31)) & 1u) continue;
      if (lane == 0) keep[nk] = (int)(key[k] & 0xFFFFFFFFu);
      nk++;
      const int q = k >> 6;
      if (lane >= q && lane < nw) {
        const unsigned long long m = mask[tri_off(k, nw) + (lane - q)];
        lo |= (unsigned)m;
        hi |= (unsigned)(m >> 32);
      }
    }
    if (lane == 0) {
      s_nkeep = nk;
      *num_keep = nk;
    }
  }
  __syncthreads();
  // (4) kept rows and combined poses (test.py:199-211)
  if (!rois_out && !poses_out) return;
  const int nk = s_nkeep;
  for (int t = threadIdx.x; t < nk * 7; t += blockDim.x) {
    const int q = t / 7, c = t % 7;
    const int i = keep[q];
    if (rois_out) rois_out[(size_t)q * 7 + c] = rois[(size_t)i * stride + c];
    if (poses_out) {
      float v = poses_init[(size_t)i * 7 + c];
      const int cls = (int)rois[(size_t)i * stride + 1];
      if (c < 4 && cls >= 0 && poses_pred && 4 * cls + 3 < pred_dim) v = poses_pred[(size_t)i * pred_dim + 4 * cls + c];
      poses_out[(size_t)q * 7 + c] = v;
    }
  }
}

}  // namespace

extern "C" int pcnn_box_nms(const float* rois, int R_cap, int roi_stride, const int32_t* num_rois_dev, float thresh,
                            int32_t* keep, int32_t* num_keep, const float* poses_init, const float* poses_pred,
                            int pred_dim, float* rois_out, float* poses_out, void* stream) {
  PCNN_REQUIRE(rois && keep && num_keep && R_cap >= 0 && R_cap <= kNmsMaxRows && roi_stride >= 7);
  PCNN_REQUIRE(!poses_out || poses_init);
  hipLaunchKernelGGL(k_box_nms, dim3(1), dim3(kNmsThreads), 0, (hipStream_t)stream, rois, R_cap, roi_stride,
                     num_rois_dev, thresh, keep, num_keep, poses_init, poses_pred, pred_dim, rois_out, poses_out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
