// Hough voting, stage 3: exact hough_data at the cells the max selection consumes.
//
// The reference computes, for every cell with votes, the mean distance of its
// voters (sum in voter order, cu.cc:269-298) and the bb extent from a second
// voter pass with T(mean distance) (cu.cc:300-330).  Only the argmax cells
// (default path, cu.cc:751-764) and the NMS candidates (cu.cc:351) ever read
// them, so this stage re-runs both voter loops exactly at those cells only:
// flags in parallel, the distance sum sequentially in voter order (bit-equal
// to the reference's per-thread loop), bb extent as an order-free max.
// The recount must equal the interval vote's count (diag[0]).
// Multi-instance path (threshold_vote > 0, compute_max_indexes_kernel
// cu.cc:335-383): 7x7 strict local maxima above the threshold, exact
// hough_data per candidate, bb > 0 and vote-percentage filter, first
// index_size in ascending flat (slot, y, x) order.
#include "hough_common.h"

namespace pcnn_hough {

struct PeakOut { float count, distance, bbh2, bbw2; int mismatch; };

// Block-wide: all threads call; returns valid values in thread 0.
__device__ PeakOut exact_cell(int cx, int cy, int cls, float count_f, const float4* __restrict__ vd,
                              const int32_t* __restrict__ vp, int nv, int W, float inlier,
                              const float* __restrict__ extents, const float* __restrict__ meta, float* sh_d,
                              float* sh_red) {
  PeakOut o;
  float dsum = 0.f;  // meaningful in thread 0
  int cnt = 0;
  for (int start = 0; start < nv; start += kPeakChunk) {
    const int n = min(kPeakChunk, nv - start);
    if (threadIdx.x < 4) sh_d[n + threadIdx.x] = 0.f;  // pad to a float4 multiple (+0.0f is exact)
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      const float4 q = vd[start + j];
      const int p = vp[start + j];
      const int x = p % W, y = p / W;
      bool f = cone_pred(cx, cy, x, y, q.x, q.y, inlier);
      if (f) {
        float dx = fabsf((float)(x - cx));
        float dy = fabsf((float)(y - cy));
        f = dx < q.w && dy < q.w;  // cu.cc:288
      }
      sh_d[j] = f ? q.z : 0.f;  // adding +0.0f leaves a non-negative sum unchanged
      cnt += f ? 1 : 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // distance += d in voter order (cu.cc:291); loads batched, adds in order
      const float4* p4 = (const float4*)sh_d;
      const int n4 = (n + 3) / 4;
      int i = 0;
      for (; i + 4 <= n4; i += 4) {
        const float4 a = p4[i], bb = p4[i + 1], cc = p4[i + 2], dd = p4[i + 3];
        dsum += a.x; dsum += a.y; dsum += a.z; dsum += a.w;
        dsum += bb.x; dsum += bb.y; dsum += bb.z; dsum += bb.w;
        dsum += cc.x; dsum += cc.y; dsum += cc.z; dsum += cc.w;
        dsum += dd.x; dsum += dd.y; dsum += dd.z; dsum += dd.w;
      }
      for (; i < n4; i++) {
        const float4 a = p4[i];
        dsum += a.x; dsum += a.y; dsum += a.z; dsum += a.w;
      }
    }
    __syncthreads();
  }
  // block reduce count
  int wc = pcnn::wave_sum(cnt);
  if (pcnn::lane_id() == 0) sh_red[threadIdx.x >> 6] = __int_as_float(wc);
  __syncthreads();
  int tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); w++) tot += __float_as_int(sh_red[w]);
  __syncthreads();
  o.mismatch = ((float)tot != count_f) ? 1 : 0;
  o.count = count_f;
  o.distance = 0.f;
  o.bbh2 = 0.f;
  o.bbw2 = 0.f;
  if (!(count_f > 0.f)) return o;  // hough_data stays memset-zero (cu.cc:296, :698-708)
  // distance broadcast from thread 0
  if (threadIdx.x == 0) sh_red[0] = dsum / count_f;  // cu.cc:298
  __syncthreads();
  const float distance = sh_red[0];
  __syncthreads();
  const float Tm = project_box(cls, extents, meta, distance, 0.6f);  // cu.cc:317
  float bbw = -1.f, bbh = -1.f;
  for (int j = threadIdx.x; j < nv; j += blockDim.x) {
    const float4 q = vd[j];
    const int p = vp[j];
    const int x = p % W, y = p / W;
    if (cone_pred(cx, cy, x, y, q.x, q.y, inlier)) {
      float dx = fabsf((float)(x - cx));
      float dy = fabsf((float)(y - cy));
      if (dx < Tm && dy < Tm) {  // cu.cc:320-323 (max is order-independent)
        bbw = fmaxf(bbw, dx);
        bbh = fmaxf(bbh, dy);
      }
    }
  }
  bbw = pcnn::wave_max(bbw);
  bbh = pcnn::wave_max(bbh);
  if (pcnn::lane_id() == 0) {
    sh_red[2 * (threadIdx.x >> 6)] = bbw;
    sh_red[2 * (threadIdx.x >> 6) + 1] = bbh;
  }
  __syncthreads();
  for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
    bbw = fmaxf(bbw, sh_red[2 * w]);
    bbh = fmaxf(bbh, sh_red[2 * w + 1]);
  }
  bbw = fmaxf(bbw, sh_red[0]);
  bbh = fmaxf(bbh, sh_red[1]);
  __syncthreads();
  o.distance = distance;
  o.bbh2 = 2 * bbh;
  o.bbw2 = 2 * bbw;
  return o;
}

__global__ void __launch_bounds__(kPeakThreads) k_hough_peak(int H, int W, int C, float inlier,
                                                              const float* __restrict__ extents,
                                                              const float* __restrict__ meta, int num_meta,
                                                              HoughWs ws) {
  __shared__ __attribute__((aligned(16))) float sh_d[kPeakChunk + 4];
  __shared__ float sh_red[16];
  const int b = blockIdx.y, slot = blockIdx.x;
  if (slot >= ws.nvote[b]) return;
  const int cls = ws.slot_cls[(size_t)b * C + slot];
  const unsigned long long key = ws.key[(size_t)b * C + slot];
  const unsigned cnt = (unsigned)(key >> 32);
  const unsigned idx = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
  const int cx = (int)(idx % (unsigned)W), cy = (int)(idx / (unsigned)W);
  const int vb = ws.vbase[(size_t)b * C + cls];
  const int nv = ws.vcount[(size_t)b * C + cls];
  PeakOut o = exact_cell(cx, cy, cls, (float)cnt, ws.vdat + (size_t)b * ws.vcap + vb,
                         ws.vpos + (size_t)b * ws.vcap + vb, nv, W, inlier, extents, meta + (size_t)b * num_meta,
                         sh_d, sh_red);
  if (threadIdx.x == 0) {
    float* pk = ws.peak + ((size_t)b * ws.pks + slot) * 8;
    pk[0] = o.count;
    pk[1] = o.distance;
    pk[2] = o.bbh2;
    pk[3] = o.bbw2;
    pk[4] = (float)cx;
    pk[5] = (float)cy;
    if (o.mismatch) atomicAdd(&ws.diag[0], 1);
  }
}

// multi-instance (NMS) path

__global__ void __launch_bounds__(256) k_hough_nms_cand(int H, int W, int C, float vote_thr, HoughWs ws) {
  const int b = blockIdx.z, slot = blockIdx.y;
  if (slot >= ws.nvote[b]) return;
  const int HW = H * W;
  const int32_t* cm = ws.counts + ((size_t)b * (C - 1) + slot) * (size_t)HW;
  for (int cell = blockIdx.x * blockDim.x + threadIdx.x; cell < HW; cell += gridDim.x * blockDim.x) {
    const int c0 = cm[cell];
    if (!((float)c0 > vote_thr)) continue;  // cu.cc:351
    const int cx = cell % W, cy = cell / W;
    bool flag = false;
    for (int x = cx - 3; x <= cx + 3 && !flag; x++)
      for (int y = cy - 3; y <= cy + 3; y++)
        if (x >= 0 && x < W && y >= 0 && y < H && cm[y * W + x] > c0) { flag = true; break; }
    if (flag) continue;
    int q = atomicAdd(&ws.ncand[b], 1);
    if (q < kCandCap) ws.cand[(size_t)b * kCandCap + q] = slot * HW + cell;
    else atomicAdd(&ws.diag[1], 1);
  }
}

__global__ void __launch_bounds__(kPeakThreads) k_hough_cand_data(int H, int W, int C, float inlier,
                                                                   const float* __restrict__ extents,
                                                                   const float* __restrict__ meta, int num_meta,
                                                                   HoughWs ws) {
  __shared__ __attribute__((aligned(16))) float sh_d[kPeakChunk + 4];
  __shared__ float sh_red[16];
  const int b = blockIdx.y;
  const int ncand = min(ws.ncand[b], kCandCap);
  const int HW = H * W;
  for (int q = blockIdx.x; q < ncand; q += gridDim.x) {
    const int flat = ws.cand[(size_t)b * kCandCap + q];
    const int slot = flat / HW, cell = flat % HW;
    const int cls = ws.slot_cls[(size_t)b * C + slot];
    const int vb = ws.vbase[(size_t)b * C + cls];
    const int nv = ws.vcount[(size_t)b * C + cls];
    const float cnt = (float)ws.counts[((size_t)b * (C - 1) + slot) * (size_t)HW + cell];
    PeakOut o = exact_cell(cell % W, cell / W, cls, cnt, ws.vdat + (size_t)b * ws.vcap + vb,
                           ws.vpos + (size_t)b * ws.vcap + vb, nv, W, inlier, extents,
                           meta + (size_t)b * num_meta, sh_d, sh_red);
    if (threadIdx.x == 0) {
      float* cd = ws.cand_data + ((size_t)b * kCandCap + q) * 4;
      cd[0] = o.count;
      cd[1] = o.distance;
      cd[2] = o.bbh2;
      cd[3] = o.bbw2;
      if (o.mismatch) atomicAdd(&ws.diag[0], 1);
    }
    __syncthreads();
  }
}

// NMS selection per image: candidates passing bb > 0 and the vote percentage
// (cu.cc:351, :369-371), first index_size in ascending flat order.  Writes the
// kept maxima into peak[b][k] (count, distance, 2bb_h, 2bb_w, cx, cy, slot).
__global__ void __launch_bounds__(1024) k_hough_nms_select(int H, int W, int C, float per_thr, int index_size,
                                                            HoughWs ws) {
  __shared__ unsigned long long keys[kCandCap];
  const int b = blockIdx.x;
  const int ncand = min(ws.ncand[b], kCandCap);
  int n2 = 1;
  while (n2 < ncand) n2 <<= 1;
  for (int i = threadIdx.x; i < n2; i += blockDim.x) {
    unsigned long long k = ~0ull;
    if (i < ncand) {
      const float* cd = ws.cand_data + ((size_t)b * kCandCap + i) * 4;
      const float cnt = cd[0], bbh = cd[2], bbw = cd[3];
      bool keep = bbh > 0 && bbw > 0 && !(cnt / (bbh * bbw) < per_thr);
      if (keep) k = ((unsigned long long)(unsigned)ws.cand[(size_t)b * kCandCap + i] << 32) | (unsigned)i;
    }
    keys[i] = k;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        int j = i ^ stride;
        if (j > i) {
          bool up = (i & size) == 0;
          unsigned long long a = keys[i], c = keys[j];
          if ((a > c) == up) { keys[i] = c; keys[j] = a; }
        }
      }
      __syncthreads();
    }
  const int HW = H * W;
  int kept = 0;
  for (int i = 0; i < n2 && i < index_size; i++) kept += keys[i] != ~0ull ? 1 : 0;
  for (int i = threadIdx.x; i < kept; i += blockDim.x) {
    const int qi = (int)(keys[i] & 0xFFFFFFFFull);
    const int flat = (int)(keys[i] >> 32);
    const float* cd = ws.cand_data + ((size_t)b * kCandCap + qi) * 4;
    float* pk = ws.peak + ((size_t)b * ws.pks + i) * 8;
    pk[0] = cd[0];
    pk[1] = cd[1];
    pk[2] = cd[2];
    pk[3] = cd[3];
    pk[4] = (float)((flat % HW) % W);
    pk[5] = (float)((flat % HW) / W);
    pk[6] = (float)(flat / HW);
  }
  if (threadIdx.x == 0) ws.nvote[b] = kept;  // number of kept maxima of this image
}

}  // namespace pcnn_hough
