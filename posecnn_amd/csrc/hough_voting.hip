// Hough voting for PoseCNN on MI355X (gfx950).
//
// Replaces HoughVotingLaucher (lib/hough_voting_gpu_layer/hough_voting_gpu_op.cu.cc:615-799)
// and the per-image loop of HoughvotinggpuOp<GPU>::Compute (hough_voting_gpu_op.cc:321-429).
//
// The reference evaluates every (present class, Hough cell, sampled voter)
// triple — O(count * H * W * N_c / skip) predicate evaluations with a global
// `hough_space[index]++` in the inner loop (cu.cc:253-294), plus ~6 host syncs
// per image.  This implementation produces the same counts with a different
// schedule and no host synchronisation:
//
//  1. k_label_hist / k_label_scan / k_label_scatter: one coalesced pass over
//     the label map builds, per image and class, the voter list in ascending
//     raster order (the canonical order of the reference's atomic compaction,
//     cu.cc:174-187), sampling list positions 0, skip, 2 skip, ...; each voter
//     gathers its (u, v, z) once and precomputes d = exp(z) and the box
//     threshold T(d) (project_box, cu.cc:84-120).
//  2. k_hough_vote: one workgroup per (row band, class slot, image).  For every
//     voter and every row of the band inside its +-T box, the set of cells
//     whose vote predicate holds (cu.cc:283-288) is an interval (the cone of
//     half-angle acos(0.9) is convex).  The interval is computed in double for
//     an outer and an inner cone (threshold -+ 2e-6, ~4x the worst-case float
//     error of the reference's predicate); cells inside the inner cone vote,
//     cells outside the outer cone do not, and the few cells between are
//     decided by evaluating the reference's float predicate itself.  Runs are
//     added to an LDS difference array (+1/-1, integer, order-free), prefix
//     summed per row, and the per-class argmax (first maximum, = thrust
//     max_element, cu.cc:757) is folded into one 64-bit atomicMax per block.
//  3. k_hough_peak: at each argmax cell the reference's two voter loops are
//     re-run exactly (distance sum in voter order, cu.cc:269-298; bb extent
//     with T(mean distance), cu.cc:300-330).  The exact re-count must equal
//     the interval count (checked, reported by pcnn_hough_voting_diag).
//  4. Multi-instance path (threshold_vote > 0, compute_max_indexes_kernel
//     cu.cc:335-383): counts are written out, k_hough_nms_cand finds the 7x7
//     local maxima above the threshold, k_hough_cand_data evaluates their
//     hough_data exactly, k_hough_emit keeps the first index_size in ascending
//     flat order.
//  5. k_hough_emit: compute_rois_kernel (cu.cc:386-576) for every kept max,
//     image-major / ascending slot order, into capacity-sized outputs with a
//     device-side row count.
#include "pcnn_common.h"
#include <math.h>

namespace {

constexpr int kMaxClasses = 256;
constexpr int kPixPerBlk = 4096;   // label pixels per compaction block
constexpr int kCompactThreads = 256;
constexpr int kBand = 8;           // Hough rows per vote workgroup
constexpr int kVoteThreads = 256;
constexpr int kPeakThreads = 256;
constexpr int kPeakChunk = 1024;   // voters per ordered-sum chunk
constexpr int kCandCap = 4096;     // NMS candidates per image
constexpr double kConeEps = 2e-6;  // margin of the exact-predicate band (in cos)

struct HoughWs {
  int32_t* blk;       // [B][NBLK][C] per-block class histogram -> exclusive offsets
  int32_t* total;     // [B][C]
  int32_t* nslots;    // [B] present classes
  int32_t* nvote;     // [B] slots voted (default: min(count, index_size); NMS: count)
  int32_t* slot_cls;  // [B][C]
  int32_t* vbase;     // [B][C] voter list offset of class c (image-relative)
  int32_t* vcount;    // [B][C] voters of class c (0 when not voted)
  float4* vdat;       // [B][VCAP] (u, v, d, T)
  int32_t* vpos;      // [B][VCAP] y*W + x
  unsigned long long* key;  // [B][C] argmax key per slot
  float* peak;        // [B][C][8] count, distance, 2bb_h, 2bb_w, cx, cy
  int32_t* counts;    // [B][C-1][H*W] (NMS path)
  int32_t* ncand;     // [B]
  int32_t* cand;      // [B][kCandCap] slot*HW + cell
  float* cand_data;   // [B][kCandCap][4] count, distance, 2bb_h, 2bb_w
  int32_t* diag;      // [4]
  int nblk, vcap, pks;  // pks = peak slots per image = max(C, PCNN_MAX_ROI)
};

HoughWs carve_ws(void* base, int B, int H, int W, int C, int skip, bool nms, size_t* total_bytes) {
  pcnn::Carve cv(base);
  HoughWs ws;
  const long HW = (long)H * W;
  ws.nblk = (int)((HW + kPixPerBlk - 1) / kPixPerBlk);
  ws.vcap = (int)((HW + skip - 1) / skip) + C;
  ws.pks = C > PCNN_MAX_ROI ? C : PCNN_MAX_ROI;
  ws.diag = cv.take<int32_t>(4);
  ws.blk = cv.take<int32_t>((size_t)B * ws.nblk * C);
  ws.total = cv.take<int32_t>((size_t)B * C);
  ws.nslots = cv.take<int32_t>(B);
  ws.nvote = cv.take<int32_t>(B);
  ws.slot_cls = cv.take<int32_t>((size_t)B * C);
  ws.vbase = cv.take<int32_t>((size_t)B * C);
  ws.vcount = cv.take<int32_t>((size_t)B * C);
  ws.vdat = cv.take<float4>((size_t)B * ws.vcap);
  ws.vpos = cv.take<int32_t>((size_t)B * ws.vcap);
  ws.key = cv.take<unsigned long long>((size_t)B * C);
  ws.peak = cv.take<float>((size_t)B * ws.pks * 8);
  ws.ncand = cv.take<int32_t>(B);
  if (nms) {
    ws.counts = cv.take<int32_t>((size_t)B * (C - 1) * HW);
    ws.cand = cv.take<int32_t>((size_t)B * kCandCap);
    ws.cand_data = cv.take<float>((size_t)B * kCandCap * 4);
  } else {
    ws.counts = nullptr;
    ws.cand = nullptr;
    ws.cand_data = nullptr;
  }
  if (total_bytes) *total_bytes = cv.off;
  return ws;
}

// ---------------------------------------------------------------------------
// Reference arithmetic (evaluated with every op rounded separately).

// angle_distance(...) > inlierThreshold (cu.cc:32-42, :283)
__device__ __forceinline__ bool cone_pred(int cx, int cy, int x, int y, float u, float v, float thr) {
  float dx = (float)(cx - x);
  float dy = (float)(cy - y);
  float n1 = sqrtf(u * u + v * v);
  float n2 = sqrtf(dx * dx + dy * dy);
  float dot = u * dx + v * dy;
  return dot / (n1 * n2) > thr;
}

// project_box (cu.cc:84-120)
__device__ float project_box(int cls, const float* __restrict__ extents, const float* __restrict__ meta,
                             float distance, float factor) {
  float xHalf = (float)((double)extents[cls * 3 + 0] * 0.5);
  float yHalf = (float)((double)extents[cls * 3 + 1] * 0.5);
  float zHalf = (float)((double)extents[cls * 3 + 2] * 0.5);
  const float fx = meta[0], fy = meta[4], px = meta[2], py = meta[5];
  const float zf = zHalf + distance, zb = -zHalf + distance;
  float minX = 1e8f, maxX = -1e8f, minY = 1e8f, maxY = -1e8f;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const float X = (i & 1) ? -xHalf : xHalf;
    const float Y = (i & 2) ? -yHalf : yHalf;
    const float Z = (i & 4) ? zb : zf;
    float x = fx * (X / Z) + px;
    float y = fy * (Y / Z) + py;
    minX = fminf(minX, x);
    minY = fminf(minY, y);
    maxX = fmaxf(maxX, x);
    maxY = fmaxf(maxY, y);
  }
  float width = maxX - minX + 1;
  float height = maxY - minY + 1;
  return fmaxf(width, height) * factor;
}

// IoU (cu.cc:73-82)
__device__ float iou4(const float* a, const float* b) {
  float left = fmaxf(a[0], b[0]), right = fminf(a[2], b[2]);
  float top = fmaxf(a[1], b[1]), bottom = fminf(a[3], b[3]);
  float width = fmaxf(right - left + 1, 0.f), height = fmaxf(bottom - top + 1, 0.f);
  float interS = width * height;
  float Sa = (a[2] - a[0] + 1) * (a[3] - a[1] + 1);
  float Sb = (b[2] - b[0] + 1) * (b[3] - b[1] + 1);
  return interS / (Sa + Sb - interS);
}

// compute_box_overlap (cu.cc:123-172); Eigen Quaternionf::toRotationMatrix,
// lazy 3x3*3x8 product summed a0 + (a1 + a2).
__device__ float box_overlap(int cls, const float* __restrict__ extents, const float* __restrict__ meta,
                             const float* __restrict__ pose, const float* box) {
  float xHalf = (float)((double)extents[cls * 3 + 0] * 0.5);
  float yHalf = (float)((double)extents[cls * 3 + 1] * 0.5);
  float zHalf = (float)((double)extents[cls * 3 + 2] * 0.5);
  float qw = pose[6], qx = pose[7], qy = pose[8], qz = pose[9];
  float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
  float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  float R[9] = {1.f - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.f - (txx + tzz), tyz - twx,
                txz - twy, tyz + twx, 1.f - (txx + tyy)};
  const float fx = meta[0], fy = meta[4], px = meta[2], py = meta[5];
  float x1 = 1e8f, x2 = -1e8f, y1 = 1e8f, y2 = -1e8f;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const float bx = (i & 1) ? -xHalf : xHalf;
    const float by = (i & 2) ? -yHalf : yHalf;
    const float bz = (i & 4) ? -zHalf : zHalf;
    float X = R[0] * bx + (R[1] * by + R[2] * bz);
    float Y = R[3] * bx + (R[4] * by + R[5] * bz);
    float Z = R[6] * bx + (R[7] * by + R[8] * bz);
    X = X + pose[10];
    Y = Y + pose[11];
    Z = Z + pose[12];
    float x = fx * (X / Z) + px;
    float y = fy * (Y / Z) + py;
    x1 = fminf(x1, x);
    y1 = fminf(y1, y);
    x2 = fmaxf(x2, x);
    y2 = fmaxf(y2, y);
  }
  float gtb[4] = {x1, y1, x2, y2};
  return iou4(box, gtb);
}

// largest integer k with k < T (the box test |dx| < T on integer dx), or -1.
__device__ __forceinline__ int box_radius(float T) {
  if (!(T > 0.f)) return -1;
  if (T > 1.0e7f) return 10000000;
  return (int)ceilf(T) - 1;
}

// Wave-aggregated grouping of lanes by label: calls fn(label, mask) once per
// distinct valid label of the wave (same label in every lane of `mask`).
template <typename F>
__device__ __forceinline__ void for_each_label_group(int lab, bool valid, F fn) {
  uint64_t active = __ballot(valid);
  while (active) {
    int leader = __ffsll((long long)active) - 1;
    int l0 = __shfl(lab, leader, 64);
    uint64_t m = __ballot(valid && lab == l0);
    fn(l0, m);
    active &= ~m;
  }
}

// ---------------------------------------------------------------------------
// 1. label compaction

__global__ void __launch_bounds__(kCompactThreads) k_label_hist(const int32_t* __restrict__ label, int HW, int C,
                                                                 HoughWs ws) {
  __shared__ int h[kMaxClasses];
  const int b = blockIdx.y, blk = blockIdx.x;
  for (int i = threadIdx.x; i < C; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int32_t* lab = label + (size_t)b * HW;
  const int base = blk * kPixPerBlk;
  for (int r = 0; r < kPixPerBlk / kCompactThreads; r++) {
    int p = base + r * kCompactThreads + threadIdx.x;
    int l = p < HW ? lab[p] : -1;
    bool valid = p < HW && l > 0 && l < C;
    for_each_label_group(l, valid, [&](int l0, uint64_t m) {
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) atomicAdd(&h[l0], __popcll(m));
    });
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) ws.blk[((size_t)b * ws.nblk + blk) * C + i] = h[i];
}

__global__ void __launch_bounds__(256) k_label_scan(int C, int label_thr, int index_size, int nms, int skip,
                                                     HoughWs ws) {
  __shared__ int tot[kMaxClasses];
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    int run = 0;
    int32_t* col = ws.blk + (size_t)b * ws.nblk * C + c;
    for (int k = 0; k < ws.nblk; k++) {
      int v = col[(size_t)k * C];
      col[(size_t)k * C] = run;
      run += v;
    }
    tot[c] = run;
    ws.total[(size_t)b * C + c] = run;
    ws.key[(size_t)b * C + c] = 0ull;
    ws.vcount[(size_t)b * C + c] = 0;
    ws.vbase[(size_t)b * C + c] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int count = 0;
    for (int c = 1; c < C; c++)  // cu.cc:654-664
      if (tot[c] > label_thr) ws.slot_cls[(size_t)b * C + count++] = c;
    int nvote = nms ? count : (count < index_size ? count : index_size);
    ws.nslots[b] = count;
    ws.nvote[b] = nvote;
    ws.ncand[b] = 0;
    int vb = 0;
    for (int s = 0; s < nvote; s++) {
      int c = ws.slot_cls[(size_t)b * C + s];
      int nv = (tot[c] + skip - 1) / skip;
      ws.vbase[(size_t)b * C + c] = vb;
      ws.vcount[(size_t)b * C + c] = nv;
      vb += nv;
    }
  }
}

__global__ void __launch_bounds__(kCompactThreads) k_label_scatter(const int32_t* __restrict__ label,
                                                                    const float* __restrict__ vertex,
                                                                    const float* __restrict__ extents,
                                                                    const float* __restrict__ meta, int num_meta,
                                                                    int H, int W, int C, int skip, HoughWs ws) {
  __shared__ int run[kMaxClasses];
  __shared__ int vc[kMaxClasses];
  __shared__ int wcnt[kCompactThreads / 64][kMaxClasses];
  const int b = blockIdx.y, blk = blockIdx.x;
  const int HW = H * W;
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    run[i] = ws.blk[((size_t)b * ws.nblk + blk) * C + i];
    vc[i] = ws.vcount[(size_t)b * C + i];
  }
  const int32_t* lab = label + (size_t)b * HW;
  const float* mb = meta + (size_t)b * num_meta;
  const int base = blk * kPixPerBlk;
  __syncthreads();
  for (int r = 0; r < kPixPerBlk / kCompactThreads; r++) {
    for (int i = pcnn::lane_id(); i < C; i += 64) wcnt[wave][i] = 0;
    int p = base + r * kCompactThreads + threadIdx.x;
    int l = p < HW ? lab[p] : -1;
    bool valid = p < HW && l > 0 && l < C;
    int rank_w = 0;
    for_each_label_group(l, valid, [&](int l0, uint64_t m) {
      if (l == l0 && valid) rank_w = __popcll(m & pcnn::lanemask_lt());
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) wcnt[wave][l0] = __popcll(m);
    });
    __syncthreads();
    if (valid && vc[l] > 0) {
      int rank = run[l] + rank_w;
      for (int w = 0; w < wave; w++) rank += wcnt[w][l];
      if (rank % skip == 0) {  // list positions 0, skip, 2 skip, ... (cu.cc:269)
        const int vi = ws.vbase[(size_t)b * C + l] + rank / skip;
        const size_t off = ((size_t)b * HW + p) * (size_t)(3 * C) + 3 * l;
        const float u = vertex[off], v = vertex[off + 1];
        const float d = (float)exp((double)vertex[off + 2]);  // cu.cc:280
        const float T = project_box(l, extents, mb, d, 0.6f);  // cu.cc:285
        ws.vdat[(size_t)b * ws.vcap + vi] = make_float4(u, v, d, T);
        ws.vpos[(size_t)b * ws.vcap + vi] = p;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C; i += blockDim.x) {
      int s = 0;
      for (int w = 0; w < kCompactThreads / 64; w++) s += wcnt[w][i];
      run[i] += s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// 2. interval vote

struct Cone {
  double mx, my, px, py;  // boundary rays rotated by -theta / +theta from the voter direction
};

__device__ __forceinline__ Cone make_cone(double ex, double ey, double c, double s) {
  Cone k;
  k.px = ex * c - ey * s;  // +theta (ccw)
  k.py = ex * s + ey * c;
  k.mx = ex * c + ey * s;  // -theta
  k.my = -ex * s + ey * c;
  return k;
}

// Open interval (lo, hi) of dx with (dx, dy) strictly inside the cone:
// cross(m, p) > 0 and cross(p, p+) > 0.  Returns false when empty.
__device__ __forceinline__ bool cone_row(const Cone& k, double dy, double& lo, double& hi) {
  lo = -1e30;
  hi = 1e30;
  // (1) -my * dx > -mx * dy
  double a1 = -k.my, b1 = -k.mx * dy;
  if (a1 > 0.0) lo = fmax(lo, b1 / a1);
  else if (a1 < 0.0) hi = fmin(hi, b1 / a1);
  else if (!(0.0 > b1)) return false;
  // (2) py * dx > px * dy
  double a2 = k.py, b2 = k.px * dy;
  if (a2 > 0.0) lo = fmax(lo, b2 / a2);
  else if (a2 < 0.0) hi = fmin(hi, b2 / a2);
  else if (!(0.0 > b2)) return false;
  return lo < hi;
}

// integer cell range [a, b] of x + dx for dx strictly inside (lo, hi), clipped
__device__ __forceinline__ void int_range(double lo, double hi, int x, int cx0, int cx1, int& a, int& b) {
  lo = fmax(lo, -1e9);
  hi = fmin(hi, 1e9);
  long la = (long)floor(lo) + 1 + x;
  long lb = (long)ceil(hi) - 1 + x;
  a = (int)(la < cx0 ? cx0 : la);
  b = (int)(lb > cx1 ? cx1 : lb);
}

__device__ __forceinline__ void add_run(int* row, int a, int b) {
  atomicAdd(&row[a], 1);
  atomicAdd(&row[b + 1], -1);
}

__global__ void __launch_bounds__(kVoteThreads) k_hough_vote(int H, int W, int C, float inlier, HoughWs ws,
                                                              int32_t* __restrict__ counts_out) {
  extern __shared__ __attribute__((aligned(16))) int diff[];  // [kBand][W + 1]
  __shared__ unsigned long long bkey[kVoteThreads / 64];
  const int b = blockIdx.z, slot = blockIdx.y, band = blockIdx.x;
  if (slot >= ws.nvote[b]) return;
  const int cls = ws.slot_cls[(size_t)b * C + slot];
  const int nv = ws.vcount[(size_t)b * C + cls];
  const int vb = ws.vbase[(size_t)b * C + cls];
  const int y0 = band * kBand;
  const int y1 = min(y0 + kBand, H);
  const int Wp = W + 1;
  for (int i = threadIdx.x; i < kBand * Wp; i += blockDim.x) diff[i] = 0;

  const double c = (double)inlier;
  const bool fast_ok = c > 0.05 && c < 0.999;
  const double co = c - kConeEps, ci = c + kConeEps;
  const double so = sqrt(1.0 - co * co), si = sqrt(1.0 - ci * ci);
  __syncthreads();

  const float4* vd = ws.vdat + (size_t)b * ws.vcap + vb;
  const int32_t* vp = ws.vpos + (size_t)b * ws.vcap + vb;
  for (int i = threadIdx.x; i < nv; i += blockDim.x) {
    const float4 q = vd[i];
    const int p = vp[i];
    const int x = p % W, y = p / W;
    const int k = box_radius(q.w);
    if (k < 0) continue;
    const int ry0 = max(y - k, y0), ry1 = min(y + k, y1 - 1);
    if (ry0 > ry1) continue;
    const int bx0 = max(x - k, 0), bx1 = min(x + k, W - 1);
    const float u = q.x, v = q.y;
    const float n1f = sqrtf(u * u + v * v);
    const bool slow = !fast_ok || !(n1f >= 1e-18f && n1f <= 1e18f);
    if (slow) {
      // exact predicate on every cell of the box rows (pathological voters only)
      for (int r = ry0; r <= ry1; r++) {
        int* row = diff + (r - y0) * Wp;
        int start = -1;
        for (int cx = bx0; cx <= bx1; cx++) {
          bool on = cone_pred(cx, r, x, y, u, v, inlier);
          if (on && start < 0) start = cx;
          if (!on && start >= 0) { add_run(row, start, cx - 1); start = -1; }
        }
        if (start >= 0) add_run(row, start, bx1);
      }
      continue;
    }
    const double ud = u, vdd = v;
    const double nd = sqrt(ud * ud + vdd * vdd);
    const double ex = ud / nd, ey = vdd / nd;
    const Cone ko = make_cone(ex, ey, co, so);
    const Cone ki = make_cone(ex, ey, ci, si);
    for (int r = ry0; r <= ry1; r++) {
      int* row = diff + (r - y0) * Wp;
      const double dy = (double)(r - y);
      double lo, hi;
      if (!cone_row(ko, dy, lo, hi)) continue;
      int oa, ob;
      int_range(lo, hi, x, bx0, bx1, oa, ob);
      if (oa > ob) continue;
      int ia = 1, ib = 0;
      if (cone_row(ki, dy, lo, hi)) {
        int_range(lo, hi, x, bx0, bx1, ia, ib);
        if (ia < oa) ia = oa;
        if (ib > ob) ib = ob;
      }
      if (ia <= ib) {
        add_run(row, ia, ib);
        // ambiguous band left of and right of the inner interval
        int start = -1;
        for (int cx = oa; cx < ia; cx++) {
          bool on = cone_pred(cx, r, x, y, u, v, inlier);
          if (on && start < 0) start = cx;
          if (!on && start >= 0) { add_run(row, start, cx - 1); start = -1; }
        }
        if (start >= 0) add_run(row, start, ia - 1);
        start = -1;
        for (int cx = ib + 1; cx <= ob; cx++) {
          bool on = cone_pred(cx, r, x, y, u, v, inlier);
          if (on && start < 0) start = cx;
          if (!on && start >= 0) { add_run(row, start, cx - 1); start = -1; }
        }
        if (start >= 0) add_run(row, start, ob);
      } else {
        int start = -1;
        for (int cx = oa; cx <= ob; cx++) {
          bool on = cone_pred(cx, r, x, y, u, v, inlier);
          if (on && start < 0) start = cx;
          if (!on && start >= 0) { add_run(row, start, cx - 1); start = -1; }
        }
        if (start >= 0) add_run(row, start, ob);
      }
    }
  }
  __syncthreads();

  // prefix-sum each row; first maximum in raster order -> 64-bit key
  const int wave = threadIdx.x >> 6, lane = pcnn::lane_id();
  const int nwaves = blockDim.x >> 6;
  unsigned long long best = 0ull;
  const int per = (W + 63) / 64;
  for (int r = y0 + wave; r < y1; r += nwaves) {
    int* row = diff + (r - y0) * Wp;
    const int c0 = lane * per, c1 = min(c0 + per, W);
    int s = 0;
    for (int cx = c0; cx < c1; cx++) s += row[cx];
    // exclusive wave scan of lane sums
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    int acc = incl - s;
    int32_t* crow = counts_out ? counts_out + (((size_t)b * (C - 1) + slot) * H + r) * (size_t)W : nullptr;
    for (int cx = c0; cx < c1; cx++) {
      acc += row[cx];
      const unsigned long long kk =
          ((unsigned long long)(unsigned)acc << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)(r * W + cx));
      best = kk > best ? kk : best;
      if (crow) crow[cx] = acc;
    }
  }
  best = pcnn::wave_max(best);
  if (lane == 0) bkey[wave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = bkey[0];
    for (int w = 1; w < nwaves; w++) m = bkey[w] > m ? bkey[w] : m;
    atomicMax(ws.key + (size_t)b * C + slot, m);
  }
}

// ---------------------------------------------------------------------------
// 3. exact hough_data at one cell (the reference's two voter loops)

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
    if (threadIdx.x == 0)
      for (int j = 0; j < n; j++) dsum += sh_d[j];  // distance += d in voter order (cu.cc:291)
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
  __shared__ float sh_d[kPeakChunk];
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

// ---------------------------------------------------------------------------
// 4. multi-instance (NMS) path

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
  __shared__ float sh_d[kPeakChunk];
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

// ---------------------------------------------------------------------------
// 5. RoI emission (compute_rois_kernel, cu.cc:386-576)

__global__ void __launch_bounds__(256) k_hough_emit(int B, int H, int W, int C, int is_train, int batch_base,
                                                     int nms, const float* __restrict__ extents,
                                                     const float* __restrict__ meta, int num_meta,
                                                     const float* __restrict__ gt, int num_gt, HoughWs ws,
                                                     float* __restrict__ top_box, float* __restrict__ top_pose,
                                                     float* __restrict__ top_target, float* __restrict__ top_weight,
                                                     int32_t* __restrict__ top_domain, int32_t* __restrict__ num_rois,
                                                     int cap) {
  extern __shared__ int row_off[];  // [B + 1]
  const int rpm = is_train ? 9 : 1;
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < B; b++) {
      row_off[b] = acc;
      acc += ws.nvote[b] * rpm;
    }
    row_off[B] = acc;
  }
  __syncthreads();
  const int total = row_off[B];
  const int PC = 4 * C;
  const int NS = ws.pks;
  for (int q = threadIdx.x; q < B * NS; q += blockDim.x) {
    const int b = q / NS, k = q % NS;
    if (k >= ws.nvote[b]) continue;
    const int r0 = row_off[b] + k * rpm;
    if (r0 + rpm > cap) { atomicAdd(&ws.diag[2], 1); continue; }
    const float* pk = ws.peak + ((size_t)b * ws.pks + k) * 8;
    const int slot = nms ? (int)pk[6] : k;
    const int cls = ws.slot_cls[(size_t)b * C + slot];
    const float score = pk[0], bb_distance = pk[1], bb_height = pk[2], bb_width = pk[3];
    const int x = (int)pk[4], y = (int)pk[5];
    const float* mb = meta + (size_t)b * num_meta;
    const float fx = mb[0], fy = mb[4], px = mb[2], py = mb[5];
    const float rx = ((float)x - px) / fx;
    const float ry = ((float)y - py) / fy;
    const int batch_index = batch_base + b;
    const double sc = 0.5 + (double)0.05f;
    float bx[4];
    bx[0] = (float)((double)x - (double)bb_width * sc);
    bx[1] = (float)((double)y - (double)bb_height * sc);
    bx[2] = (float)((double)x + (double)bb_width * sc);
    bx[3] = (float)((double)y + (double)bb_height * sc);
    // target / weight (train only): first same-(b, cls) GT with overlap > 0.2
    int gsel = -1;
    if (is_train) {
      for (int i = 0; i < num_gt; i++) {
        const int gt_batch = (int)gt[i * 13 + 0];
        const int gt_id = (int)gt[i * 13 + 1];
        if (cls == gt_id && batch_index == gt_batch) {
          float ov = box_overlap(cls, extents, mb, gt + (size_t)i * 13, bx);
          if ((double)ov > 0.2) { gsel = i; break; }
        }
      }
    }
    const float ww = bx[2] - bx[0], hh = bx[3] - bx[1];
    const int jit[9][2] = {{0, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}, {0, -1}, {-1, 0}, {0, 1}, {1, 0}};
    for (int j = 0; j < rpm; j++) {
      const int r = r0 + j;
      float* bo = top_box + (size_t)r * 7;
      bo[0] = (float)batch_index;
      bo[1] = (float)cls;
      if (j == 0) {
        bo[2] = bx[0]; bo[3] = bx[1]; bo[4] = bx[2]; bo[5] = bx[3];
      } else {
        const int jx = jit[j][0], jy = jit[j][1];
        const float nx = jx == 0 ? bx[0] : (float)((double)bx[0] + (jx < 0 ? -0.05 : 0.05) * (double)ww);
        const float ny = jy == 0 ? bx[1] : (float)((double)bx[1] + (jy < 0 ? -0.05 : 0.05) * (double)hh);
        bo[2] = nx;
        bo[3] = ny;
        bo[4] = nx + ww;
        bo[5] = ny + hh;
      }
      bo[6] = score;
      float* po = top_pose + (size_t)r * 7;
      po[0] = 1.f; po[1] = 0.f; po[2] = 0.f; po[3] = 0.f;
      po[4] = rx * bb_distance;
      po[5] = ry * bb_distance;
      po[6] = bb_distance;
      top_domain[r] = is_train ? (num_gt == 0 ? 1 : 0) : 0;
      float* to = top_target + (size_t)r * PC;
      float* wo = top_weight + (size_t)r * PC;
      for (int t = 0; t < PC; t++) { to[t] = 0.f; wo[t] = 0.f; }
      if (gsel >= 0)
        for (int t = 0; t < 4; t++) {
          to[4 * cls + t] = gt[gsel * 13 + 6 + t];
          wo[4 * cls + t] = 1.f;
        }
    }
  }
  if (threadIdx.x == 0) {
    const int n = total < cap ? total : cap;
    num_rois[0] = n;
    num_rois[1] = n > 0 ? n : 1;
  }
  if (total == 0) {  // dummy all-zero row (hough_voting_gpu_op.cc:382-383)
    for (int t = threadIdx.x; t < 7; t += blockDim.x) { top_box[t] = 0.f; top_pose[t] = 0.f; }
    for (int t = threadIdx.x; t < PC; t += blockDim.x) { top_target[t] = 0.f; top_weight[t] = 0.f; }
    if (threadIdx.x == 0) top_domain[0] = 0;
  }
}

__global__ void k_zero_f32(float* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

}  // namespace

extern "C" size_t pcnn_hough_voting_workspace_size(int B, int H, int W, int C, int skip_pixels, float vote_thr) {
  if (B <= 0 || H <= 0 || W <= 0 || C < 2 || skip_pixels <= 0) return 0;
  size_t bytes = 0;
  carve_ws(nullptr, B, H, W, C, skip_pixels, vote_thr > 0.f, &bytes);
  return bytes + 256;
}

extern "C" int pcnn_hough_voting(const int32_t* label, const float* vertex, const float* extents, const float* meta,
                                 int num_meta, const float* gt, int num_gt, int B, int H, int W, int C,
                                 int batch_base, int global_batch, int is_train, float inlier_thr, int label_thr,
                                 float vote_thr, float per_thr, int skip_pixels, float* top_box, float* top_pose,
                                 float* top_target, float* top_weight, int32_t* top_domain, int32_t* num_rois,
                                 int cap, int32_t* debug_counts, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C >= 2 && C <= kMaxClasses && skip_pixels > 0 && num_meta >= 6);
  PCNN_REQUIRE((long)H * W * (C - 1) < (1l << 31) && W < (1 << 16));
  PCNN_REQUIRE(label && vertex && extents && meta && top_box && top_pose && top_target && top_weight &&
               top_domain && num_rois && workspace && cap > 0);
  PCNN_REQUIRE(num_gt == 0 || gt);
  if (global_batch <= 0) global_batch = B;
  PCNN_REQUIRE(global_batch >= B);
  const bool nms = vote_thr > 0.f;
  size_t need = 0;
  carve_ws(nullptr, B, H, W, C, skip_pixels, nms, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  HoughWs ws = carve_ws(workspace, B, H, W, C, skip_pixels, nms, nullptr);
  hipStream_t st = (hipStream_t)stream;
  const int index_size = PCNN_MAX_ROI / global_batch;  // cu.cc:734

  if (hipMemsetAsync(ws.diag, 0, 4 * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  hipLaunchKernelGGL(k_label_hist, dim3(ws.nblk, B), dim3(kCompactThreads), 0, st, label, H * W, C, ws);
  hipLaunchKernelGGL(k_label_scan, dim3(B), dim3(256), 0, st, C, label_thr, index_size, nms ? 1 : 0, skip_pixels,
                     ws);
  hipLaunchKernelGGL(k_label_scatter, dim3(ws.nblk, B), dim3(kCompactThreads), 0, st, label, vertex, extents, meta,
                     num_meta, H, W, C, skip_pixels, ws);
  PCNN_CHECK_LAUNCH();
  int32_t* counts_out = nms ? ws.counts : debug_counts;
  const size_t lds = (size_t)kBand * (W + 1) * sizeof(int);
  hipLaunchKernelGGL(k_hough_vote, dim3((H + kBand - 1) / kBand, C - 1, B), dim3(kVoteThreads), lds, st, H, W, C,
                     inlier_thr, ws, counts_out);
  PCNN_CHECK_LAUNCH();
  if (!nms) {
    hipLaunchKernelGGL(k_hough_peak, dim3(C - 1, B), dim3(kPeakThreads), 0, st, H, W, C, inlier_thr, extents, meta,
                       num_meta, ws);
  } else {
    const int HW = H * W;
    hipLaunchKernelGGL(k_hough_nms_cand, dim3((HW + 255) / 256 < 64 ? (HW + 255) / 256 : 64, C - 1, B), dim3(256),
                       0, st, H, W, C, vote_thr, ws);
    hipLaunchKernelGGL(k_hough_cand_data, dim3(128, B), dim3(kPeakThreads), 0, st, H, W, C, inlier_thr, extents,
                       meta, num_meta, ws);
    hipLaunchKernelGGL(k_hough_nms_select, dim3(B), dim3(1024), 0, st, H, W, C, per_thr, index_size, ws);
    if (debug_counts &&
        hipMemcpyAsync(debug_counts, ws.counts, (size_t)B * (C - 1) * HW * sizeof(int32_t), hipMemcpyDeviceToDevice,
                       st) != hipSuccess)
      return PCNN_EHIP;
  }
  PCNN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_hough_emit, dim3(1), dim3(256), (B + 1) * sizeof(int), st, B, H, W, C, is_train, batch_base,
                     nms ? 1 : 0, extents, meta, num_meta, gt, num_gt, ws, top_box, top_pose, top_target,
                     top_weight, top_domain, num_rois, cap);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hough_voting_grad(float* grad_label, float* grad_vertex, int B, int H, int W, int C,
                                      void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0);
  hipStream_t st = (hipStream_t)stream;
  if (grad_label && hipMemsetAsync(grad_label, 0, (size_t)B * H * W * sizeof(float), st) != hipSuccess)
    return PCNN_EHIP;
  if (grad_vertex && hipMemsetAsync(grad_vertex, 0, (size_t)B * H * W * 3 * C * sizeof(float), st) != hipSuccess)
    return PCNN_EHIP;
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hough_voting_diag(const void* workspace, int B, int H, int W, int C, int skip_pixels,
                                      float vote_thr, int32_t* diag_host4, void* stream) {
  PCNN_REQUIRE(workspace && diag_host4);
  HoughWs ws = carve_ws((void*)workspace, B, H, W, C, skip_pixels, vote_thr > 0.f, nullptr);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemcpyAsync(diag_host4, ws.diag, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
    return PCNN_EHIP;
  if (hipStreamSynchronize(st) != hipSuccess) return PCNN_EHIP;
  return PCNN_OK;
}
