// Shared state and reference arithmetic of the Hough-voting op (see
// hough_emit.hip for the op overview).  Split across translation units:
//   hough_compact.hip  label histogram / scan / voter compaction
//   hough_vote.hip     interval vote into LDS difference arrays + argmax key
//   hough_peak.hip     exact hough_data at maxima, multi-instance NMS
//   hough_emit.hip     RoI emission + the C-ABI entry points
#pragma once
#include "pcnn_common.h"
#include <math.h>

namespace pcnn_hough {

constexpr int kMaxClasses = 256;
#ifndef PCNN_PIXBLK
#define PCNN_PIXBLK 2048
#endif
constexpr int kPixPerBlk = PCNN_PIXBLK;   // label pixels per compaction block
constexpr int kCompactThreads = 256;
#ifndef PCNN_PTHREADS
#define PCNN_PTHREADS 1024
#endif
constexpr int kPeakThreads = PCNN_PTHREADS;
constexpr int kPeakChunk = 4096;   // voters per ordered-sum chunk (LDS floats)
constexpr int kCandCap = 4096;     // NMS candidates per image
constexpr int kEmitThreads = 256;
constexpr double kConeEps = 2e-6;  // margin of the exact-predicate band (in cos)

// per-voter row-bound codes (2 bits per bound, 4 bounds: outer s1, s2, inner s1, s2)
constexpr int kBoundLower = 0, kBoundUpper = 1, kNeedPosDy = 2, kNeedNegDy = 3;
constexpr int kSlowVoter = 1 << 16;   // evaluate the exact predicate on every box cell
constexpr int kDeadVoter = 1 << 17;   // votes for no cell (T <= 0 or NaN)

struct HoughWs {
  int32_t* blk;       // [B][NBLK][C] per-block class histogram -> exclusive offsets
  int32_t* total;     // [B][C]
  int32_t* nslots;    // [B] present classes
  int32_t* nvote;     // [B] slots voted (default: min(count, index_size)); after NMS: kept maxima
  int32_t* nvtot;     // [B] voters of the voted slots
  int32_t* slot_cls;  // [B][C]
  int32_t* vbase;     // [B][C] voter list offset of class c (image-relative)
  int32_t* vcount;    // [B][C] voters of class c (0 when not voted)
  float4* vdat;       // [B][VCAP] (u, v, d, T)
  int32_t* vpos;      // [B][VCAP] y*W + x
  float4* vcone;      // [B][VCAP] row-bound slopes (outer s1, s2, inner s1, s2), |s| <= 1e30
  int32_t* vcode;     // [B][VCAP] bound codes | kSlowVoter | kDeadVoter
  unsigned long long* key;  // [B][C] argmax key per slot
  int32_t* rowcnt;    // [B][C][H] per slot: sampled voters in row y (the list is raster-ordered)
  int32_t* kmax;      // [B][C] per slot: largest box radius of its voters
  float* peak;        // [B][PKS][8] count, distance, 2bb_h, 2bb_w, cx, cy, slot
  int32_t* counts;    // [B][C-1][H*W] (NMS path)
  int32_t* ncand;     // [B]
  int32_t* cand;      // [B][kCandCap] slot*HW + cell
  float* cand_data;   // [B][kCandCap][4] count, distance, 2bb_h, 2bb_w
  int32_t* diag;      // [4]
  int nblk, vcap, pks;  // pks = peak slots per image = max(C, PCNN_MAX_ROI)
};

inline HoughWs carve_ws(void* base, int B, int H, int W, int C, int skip, bool nms, size_t* total_bytes) {
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
  ws.nvtot = cv.take<int32_t>(B);
  ws.slot_cls = cv.take<int32_t>((size_t)B * C);
  ws.vbase = cv.take<int32_t>((size_t)B * C);
  ws.vcount = cv.take<int32_t>((size_t)B * C);
  ws.vdat = cv.take<float4>((size_t)B * ws.vcap);
  ws.vpos = cv.take<int32_t>((size_t)B * ws.vcap);
  ws.vcone = cv.take<float4>((size_t)B * ws.vcap);
  ws.vcode = cv.take<int32_t>((size_t)B * ws.vcap);
  ws.key = cv.take<unsigned long long>((size_t)B * C);
  ws.rowcnt = cv.take<int32_t>((size_t)B * C * H);
  ws.kmax = cv.take<int32_t>((size_t)B * C);
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
// Reference arithmetic (every float op rounded separately, -ffp-contract=off).

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
__device__ __forceinline__ float project_box(int cls, const float* __restrict__ extents,
                                             const float* __restrict__ meta, float distance, float factor) {
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
__device__ __forceinline__ float iou4(const float* a, const float* b) {
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
__device__ __forceinline__ float box_overlap(int cls, const float* __restrict__ extents,
                                             const float* __restrict__ meta, const float* __restrict__ pose,
                                             const float* box) {
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

// ---------------------------------------------------------------------------
// RoI rows of one kept maximum (compute_rois_kernel, cu.cc:386-576), written
// by all threads of the calling workgroup: `rpm` rows (9 in train mode) from
// output row r0.  Box = x -+ bb * (0.5 + 0.05) in double (cu.cc:417-420);
// pose from the mean distance (cu.cc:404-410); train mode: the first
// same-(image, class) GT whose projected box overlaps > 0.2 (cu.cc:440-466,
// found as a min over the qualifying GT indices) sets targets / weights on
// all rows, 8 jittered boxes of 0.05 w/h (cu.cc:468-554), domain = (no GT).
struct EmitShared {
  float box[4], pose[3];
  int gsel;
};

__device__ __forceinline__ void emit_max(EmitShared& sh, int r0, int cap, int batch_index, int cls, float score,
                                         float bb_distance, float bb_height, float bb_width, int x, int y,
                                         int is_train, int C, const float* __restrict__ ext_cls,
                                         const float* __restrict__ mb, const float* __restrict__ gt, int num_gt,
                                         float* __restrict__ top_box, float* __restrict__ top_pose,
                                         float* __restrict__ top_target, float* __restrict__ top_weight,
                                         int32_t* __restrict__ top_domain, int32_t* __restrict__ diag) {
  const int rpm = is_train ? 9 : 1;
  const int PC = 4 * C;
  if (threadIdx.x == 0) {
    const float fx = mb[0], fy = mb[4], px = mb[2], py = mb[5];
    const float rx = ((float)x - px) / fx;  // cu.cc:404-405
    const float ry = ((float)y - py) / fy;
    const double sc = 0.5 + (double)0.05f;
    sh.box[0] = (float)((double)x - (double)bb_width * sc);
    sh.box[1] = (float)((double)y - (double)bb_height * sc);
    sh.box[2] = (float)((double)x + (double)bb_width * sc);
    sh.box[3] = (float)((double)y + (double)bb_height * sc);
    sh.pose[0] = rx * bb_distance;
    sh.pose[1] = ry * bb_distance;
    sh.pose[2] = bb_distance;
    sh.gsel = 0x7fffffff;
  }
  __syncthreads();
  if (is_train) {
    for (int i = threadIdx.x; i < num_gt; i += blockDim.x) {
      const int gt_batch = (int)gt[i * 13 + 0];
      const int gt_id = (int)gt[i * 13 + 1];
      if (cls == gt_id && batch_index == gt_batch) {
        const float ov = box_overlap(0, ext_cls, mb, gt + (size_t)i * 13, sh.box);  // ext_cls: this class's row
        if ((double)ov > 0.2) atomicMin(&sh.gsel, i);
      }
    }
  }
  __syncthreads();
  const int g = sh.gsel == 0x7fffffff ? -1 : sh.gsel;
  // jitter order of cu.cc:476-554: (0,0) then (-,-) (+,-) (-,+) (+,+) (0,-) (-,0) (0,+) (+,0)
  const int jx[9] = {0, -1, 1, -1, 1, 0, -1, 0, 1};
  const int jy[9] = {0, -1, -1, 1, 1, -1, 0, 1, 0};
  for (int j = threadIdx.x; j < rpm; j += blockDim.x) {
    const int r = r0 + j;
    if (r >= cap) {
      atomicAdd(&diag[2], 1);
      continue;
    }
    float* bo = top_box + (size_t)r * 7;
    const float x1 = sh.box[0], y1 = sh.box[1];
    bo[0] = (float)batch_index;
    bo[1] = (float)cls;
    if (j == 0) {
      bo[2] = x1; bo[3] = y1; bo[4] = sh.box[2]; bo[5] = sh.box[3];
    } else {
      const float ww = sh.box[2] - x1, hh = sh.box[3] - y1;
      const float nx = jx[j] == 0 ? x1 : (float)((double)x1 + (jx[j] < 0 ? -0.05 : 0.05) * (double)ww);
      const float ny = jy[j] == 0 ? y1 : (float)((double)y1 + (jy[j] < 0 ? -0.05 : 0.05) * (double)hh);
      bo[2] = nx;
      bo[3] = ny;
      bo[4] = nx + ww;
      bo[5] = ny + hh;
    }
    bo[6] = score;
    float* po = top_pose + (size_t)r * 7;
    po[0] = 1.f; po[1] = 0.f; po[2] = 0.f; po[3] = 0.f;
    po[4] = sh.pose[0];
    po[5] = sh.pose[1];
    po[6] = sh.pose[2];
    top_domain[r] = is_train ? (num_gt == 0 ? 1 : 0) : 0;
  }
  const int ncol = rpm * PC;
  for (int idx = threadIdx.x; idx < ncol; idx += blockDim.x) {
    const int j = idx / PC, col = idx % PC;
    const int r = r0 + j;
    if (r >= cap) continue;
    const bool on = g >= 0 && col >= 4 * cls && col < 4 * cls + 4;
    top_target[(size_t)r * PC + col] = on ? gt[g * 13 + 6 + (col - 4 * cls)] : 0.f;
    top_weight[(size_t)r * PC + col] = on ? 1.f : 0.f;
  }
}

// Row count (+ the dummy all-zero row when no RoI, hough_voting_gpu_op.cc:382-383).
__device__ __forceinline__ void emit_count(int total, int cap, int C, float* __restrict__ top_box,
                                           float* __restrict__ top_pose, float* __restrict__ top_target,
                                           float* __restrict__ top_weight, int32_t* __restrict__ top_domain,
                                           int32_t* __restrict__ num_rois) {
  const int PC = 4 * C;
  if (threadIdx.x == 0) {
    const int n = total < cap ? total : cap;
    num_rois[0] = n;
    num_rois[1] = n > 0 ? n : 1;
  }
  if (total == 0) {
    for (int t = threadIdx.x; t < 7; t += blockDim.x) {
      top_box[t] = 0.f;
      top_pose[t] = 0.f;
    }
    for (int t = threadIdx.x; t < PC; t += blockDim.x) {
      top_target[t] = 0.f;
      top_weight[t] = 0.f;
    }
    if (threadIdx.x == 0) top_domain[0] = 0;
  }
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
// Label producer: label_2d = argmax over the class axis
// of prob_normalized (B,H,W,C) fp32 (`argmax_2d`, lib/networks/network.py:
// 433-434, fed from vgg16_convs.py:144-146).  tf.argmax = numpy argmax: the
// first maximum wins; a NaN wins at its first occurrence.
constexpr int kArgmaxStagedMaxC = 96;  // classes staged through LDS per wave (64 px * C * 4 B)

__device__ __forceinline__ int argmax_classes(const float* v, int C) {
  float bv = v[0];
  if (bv != bv) return 0;
  int best = 0;
  for (int c = 1; c < C; c++) {
    const float x = v[c];
    if (x != x) return c;
    if (x > bv) { bv = x; best = c; }
  }
  return best;
}

// argmax of pixel p0 + lane of the wave's 64-pixel group [p0, p0 + 64) of one
// image's prob rows (img = prob + b*HW*C).  C <= kArgmaxStagedMaxC: the
// group's 64*C contiguous floats are read coalesced (float4 when the group is
// whole) into the wave's LDS slice `stage` and each lane scans its own row
// there; larger C reads the row from global memory directly.  Returns -1 for
// lanes past HW.  Every thread of the workgroup calls it together (it
// synchronises the workgroup around the staging).
__device__ __forceinline__ int wave_argmax_rows(const float* __restrict__ img, int p0, int HW, int C,
                                                float* stage) {
  const int lane = pcnn::lane_id();
  const int p = p0 + lane;
  if (C > kArgmaxStagedMaxC) return p < HW ? argmax_classes(img + (size_t)p * C, C) : -1;  // uniform branch
  const int npx = HW - p0 < 64 ? (HW - p0 > 0 ? HW - p0 : 0) : 64;
  const int n = npx * C;
  const float* src = img + (size_t)p0 * C;
  if (npx == 64 && ((((uintptr_t)src) & 15) == 0)) {
    const float4* s4 = (const float4*)src;
    for (int i = lane; i < n / 4; i += 64) ((float4*)stage)[i] = s4[i];
  } else {
    for (int i = lane; i < n; i += 64) stage[i] = src[i];
  }
  __syncthreads();
  const int l = p < HW ? argmax_classes(stage + lane * C, C) : -1;
  __syncthreads();  // the slice is reused by the wave's next group
  return l;
}

// ---------------------------------------------------------------------------
// kernels (defined in the TUs listed above)
__global__ void k_label_hist(const int32_t* __restrict__ label, int HW, int C, int H, HoughWs ws);
__global__ void k_label_hist_prob(const float* __restrict__ prob, int32_t* __restrict__ label_out, int HW, int C,
                                  int H, HoughWs ws);
// k_label_place's sampled voters per block: a class's pixels in a block hold
// consecutive list ranks, so it samples at most cnt / skip + 1 of them
__host__ __device__ inline int place_queue_cap(int C, int skip) {
  const int q = kPixPerBlk / skip + C + 1;
  return q < kPixPerBlk ? q : kPixPerBlk;
}
// k_label_place's static LDS (its kMaxClasses / kCompactThreads tables and
// scalars), an upper bound checked against the kernel in hough_compact.hip
constexpr size_t kPlaceStaticLds = (7 * kMaxClasses + 2 * kCompactThreads + 16) * sizeof(int);
__host__ __device__ inline size_t place_lds_bytes(int C, int skip) {
  return ((size_t)(kPixPerBlk / 64) * C + 3 * (size_t)place_queue_cap(C, skip)) * sizeof(int);
}
__global__ void k_label_place(const int32_t* __restrict__ label, const float* __restrict__ vertex, int vch,
                              const float* __restrict__ extents, const float* __restrict__ meta, int num_meta, int H,
                              int W, int C, int skip, int label_thr, int index_size, int nms, float inlier,
                              double so, double si, HoughWs ws);
template <int kBand, int kVoteThreads>
__global__ void k_hough_vote(int H, int W, int C, float inlier, HoughWs ws, int32_t* __restrict__ counts_out);
__global__ void k_hough_peak(int B, int H, int W, int C, float inlier, const float* __restrict__ extents,
                             const float* __restrict__ meta, int num_meta, HoughWs ws, int is_train, int batch_base,
                             const float* __restrict__ gt, int num_gt, float* __restrict__ top_box,
                             float* __restrict__ top_pose, float* __restrict__ top_target,
                             float* __restrict__ top_weight, int32_t* __restrict__ top_domain,
                             int32_t* __restrict__ num_rois, int cap, int psum);
__global__ void k_hough_nms_cand(int H, int W, int C, float vote_thr, HoughWs ws);
__global__ void k_hough_cand_data(int H, int W, int C, float inlier, const float* __restrict__ extents,
                                  const float* __restrict__ meta, int num_meta, HoughWs ws, int psum);
__global__ void k_hough_nms_select(int H, int W, int C, float per_thr, int index_size, HoughWs ws);

}  // namespace pcnn_hough
