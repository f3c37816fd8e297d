// ADD / ADD-S pose loss for PoseCNN on MI355X (gfx950).
//
// Replaces AveragedistanceForwardLaucher / AveragedistanceBackwardLaucher
// (lib/average_distance_loss/average_distance_loss_op_gpu.cu.cc:34-377).
//
// The reference runs one thread per (row, point), re-deriving the row's six
// 3x3 matrices per point into a (R, P, 54) global scratch and the per-point
// gradient into a (R, P, 4C) scratch (~0.64 GB at R = 432), sums both
// sequentially per row, and reduces the row losses with thrust + a host copy.
//
// Here a workgroup owns (row, chunk of kPts points), one lane per point: the
// matrices live in registers; for symmetric classes the GT-rotated model
// points are staged once per workgroup in LDS (float4) and each lane scans
// them in index order as wave-uniform broadcasts (cu.cc:150-172, first
// minimum, strict <) — the reference's per-point loop, vectorised over points.  Per-point loss and the four gradient terms use
// the reference's expressions and operation order (cu.cc:174-203) and are
// reduced in a fixed tree -> (R, chunks, 5) partials; one workgroup folds the
// partials per row and the rows into the scalar loss, in fixed order
// (deterministic; fp32 sums agree with the reference's sequential sums to
// ~1e-6 relative).
#include "pcnn_common.h"
#include "head_common.h"
#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

#ifndef ADD_LANES
#define ADD_LANES 64
#endif
constexpr int kSymLanes = ADD_LANES;           // symmetric rows: lanes per candidate group
#ifndef ADD_GRID
#define ADD_GRID 1024
#endif
#ifndef ADD_PPL
#define ADD_PPL 4
#endif
constexpr int kPPL = ADD_PPL;                  // query points per lane (independent min chains)
constexpr int kPts = kSymLanes * kPPL;         // query points per (row, chunk) item
constexpr int kMaxPointsLds = 8192;            // float4 candidates in LDS (128 KB)

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

// x / b correctly rounded, for a b fixed per launch (the loss normaliser),
// from r = RN(1 / b): y0 = RN(x r) is within ~2 ulp of x / b; one fma
// correction y1 = RN(y0 + r (x - b y0)) leaves a relative error of ~2u^2 on
// top of its own rounding, so y1 is a faithful quotient; then its remainder
// x - b y1 is exact in one fma and RN(y1 + r (x - b y1)) is the correctly
// rounded x / b (Markstein's theorem: faithful y, r = RN(1/b), no underflow
// at these magnitudes) -- the reference's IEEE division (cu.cc:181,196-202)
// in five instructions instead of the ten of the generic division sequence.
// (One correction from y0 alone is not enough: y0 need not be faithful when
// x / b has its mantissa near 2.)  pcnn_div_rn_check exposes it to the tests.
// Same for the double form.
__device__ __forceinline__ float div_rn(float x, float b, float r) {
  const float y0 = x * r;
  const float y1 = fmaf(fmaf(-y0, b, x), r, y0);
  return fmaf(fmaf(-y1, b, x), r, y1);
}
__device__ __forceinline__ double div_rn(double x, double b, double r) {
  const double y0 = x * r;
  const double y1 = fma(fma(-y0, b, x), r, y0);
  return fma(fma(-y1, b, x), r, y1);
}

__global__ void k_div_rn_check(const float* __restrict__ x, float b, int n, int dbl, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (dbl) {
    const double bd = (double)b, rd = 1.0 / bd;
    out[i] = (float)div_rn((double)x[i], bd, rd);
  } else {
    out[i] = div_rn(x[i], b, 1.f / b);
  }
}

__device__ __forceinline__ int row_class(const float* __restrict__ weight, int n, int C) {
  // first class with weight > 0 (cu.cc:47-52); the row's weights are loaded
  // eight at a time with independent loads, not one dependent load per class
  const float* w = weight + (size_t)n * 4 * C;
  for (int i0 = 0; i0 < C; i0 += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = i0 + j < C ? w[4 * (i0 + j)] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (v[j] > 0) return i0 + j;
  }
  return -1;
}

// Non-symmetric rows (and rows without weight): one workgroup per row, points
// strided over the threads; the per-point arithmetic is k_add_rows' (cu.cc:140-203).
// Run as the tail items of k_add_rows' queue, after the symmetric items, so
// they fill the workgroups that finish the O(P^2) items early.
__device__ __forceinline__ void add_plain_row(int n, const float* __restrict__ pred, const float* __restrict__ target,
                                              const float* __restrict__ points, const float* __restrict__ symmetry,
                                              int R, int C, int P, float margin, int norm_rows,
                                              const int32_t* __restrict__ norm_rows_dev, int nchunk,
                                              const int32_t* __restrict__ rcls, float* __restrict__ partial,
                                              float (*red)[5]) {
  const int cls = rcls[n];
  if (cls >= 0 && symmetry[cls] > 0) return;  // the symmetric items own this row
  float* out = partial + (size_t)n * nchunk * 5;
  for (int i = threadIdx.x; i < nchunk * 5; i += blockDim.x) out[i] = 0.f;
  if (cls < 0) return;
  const int PC = 4 * C;
  const float* tq = target + (size_t)n * PC + 4 * cls;
  const float* pq = pred + (size_t)n * PC + 4 * cls;
  float Rg[9], Rp[9];
  quat2rot(tq[0], tq[1], tq[2], tq[3], Rg);
  const float s = pq[0], u = pq[1], v = pq[2], w = pq[3];
  quat2rot(s, u, v, w, Rp);
  const float d0[9] = {2 * s, -2 * w, 2 * v, 2 * w, 2 * s, -2 * u, -2 * v, 2 * u, 2 * s};
  const float d1[9] = {2 * u, 2 * v, 2 * w, 2 * v, -2 * u, -2 * s, 2 * w, 2 * s, -2 * u};
  const float d2[9] = {-2 * v, 2 * u, 2 * s, 2 * u, 2 * v, 2 * w, -2 * s, 2 * w, -2 * v};
  const float d3[9] = {-2 * w, -2 * s, 2 * u, 2 * s, -2 * w, 2 * v, 2 * u, 2 * v, 2 * w};
  const int Rn = norm_rows_dev ? *norm_rows_dev : (norm_rows > 0 ? norm_rows : R);
  const float bn = (float)(Rn * P), rbn = 1.f / bn;
  const double ln = 2.0 * (double)Rn * (double)P, rln = 1.0 / ln;
  const float* pts = points + (size_t)cls * P * 3;
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const float X0 = pts[p * 3 + 0], X1 = pts[p * 3 + 1], X2 = pts[p * 3 + 2];
    const float x1 = Rp[0] * X0 + Rp[1] * X1 + Rp[2] * X2;
    const float y1 = Rp[3] * X0 + Rp[4] * X1 + Rp[5] * X2;
    const float z1 = Rp[6] * X0 + Rp[7] * X1 + Rp[8] * X2;
    const float x2 = Rg[0] * X0 + Rg[1] * X1 + Rg[2] * X2;
    const float y2 = Rg[3] * X0 + Rg[4] * X1 + Rg[5] * X2;
    const float z2 = Rg[6] * X0 + Rg[7] * X1 + Rg[8] * X2;
    const float dist = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2);
    if (dist < margin) continue;
    acc[0] += (float)div_rn((double)(dist - margin), ln, rln);
    const float X[3] = {X0, X1, X2};
    const float df[3] = {x1 - x2, y1 - y2, z1 - z2};
    float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;  // this point's terms, reference order
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        e0 += div_rn(df[j] * X[k] * d0[j * 3 + k], bn, rbn);
        e1 += div_rn(df[j] * X[k] * d1[j * 3 + k], bn, rbn);
        e2 += div_rn(df[j] * X[k] * d2[j * 3 + k], bn, rbn);
        e3 += div_rn(df[j] * X[k] * d3[j * 3 + k], bn, rbn);
      }
    acc[1] += e0; acc[2] += e1; acc[3] += e2; acc[4] += e3;
  }
#pragma unroll
  for (int q = 0; q < 5; q++) acc[q] = pcnn::wave_sum(acc[q]);
  if (pcnn::lane_id() == 0)
    for (int q = 0; q < 5; q++) red[threadIdx.x >> 6][q] = acc[q];
  __syncthreads();
  if (threadIdx.x < 5) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i][threadIdx.x];
    out[threadIdx.x] = t;
  }
}

// Symmetric rows: a 256-thread workgroup owns (row, chunk of kPts = 256 query
// points); its four one-wave groups scan disjoint quarters of the candidate
// list for the same query points (kPPL = 4 chains per lane: each broadcast
// candidate read serves four distances), then merge in LDS in group order
// with a strict < — a later range wins only with a strictly smaller
// distance, which is exactly the reference's sequential first minimum
// (cu.cc:150-172).  Round 6 geometry sweep of the whole op on the bench's
// rows (scripts/add_bench.py, one box, profiles/r06/add_geometry_sweep.log):
// 8 groups / 768 workgroups 143-148 us; 4 groups 126-130 us (kept, with a
// 1024-workgroup grid: 124-130 us); kPPL 2 129-134 us; 16 groups, kPPL 8,
// blocks of 16: slower.  Half the workgroup, twice as many in flight: the
// merge and per-item staging cost less, and more items overlap the scans.
#ifndef ADD_GROUPS
#define ADD_GROUPS 4
#endif
constexpr int kSymGroups = ADD_GROUPS;
constexpr int kSymThreads = kSymLanes * kSymGroups;
#ifndef ADD_BLK
#define ADD_BLK 8
#endif
constexpr int kBlk = ADD_BLK;  // candidates per block of the running-minimum scan

__global__ void __launch_bounds__(kSymThreads) k_add_rows(const float* __restrict__ pred,
                                                           const float* __restrict__ target,
                                                           const float* __restrict__ weight,
                                                           const float* __restrict__ points,
                                                           const float* __restrict__ symmetry, int R_cap,
                                                           const int32_t* __restrict__ num_rois_dev, int C, int P,
                                                           float margin, int norm_rows,
                                                           const int32_t* __restrict__ norm_rows_dev, int nchunk,
                                                           const int32_t* __restrict__ rcls,
                                                           const int32_t* __restrict__ sym_rows,
                                                           const int32_t* __restrict__ nsym,
                                                           int32_t* __restrict__ queue,
                                                           float* __restrict__ partial,
                                                           const int32_t* __restrict__ nearest_in,
                                                           const int32_t* __restrict__ perm_ok) {
  extern __shared__ __attribute__((aligned(16))) float4 gpts[];  // [P] GT-rotated points
  __shared__ float mdist[kSymGroups - 1][kPts];                   // range minima of groups 1..kSymGroups-1
  __shared__ int midx[kSymGroups - 1][kPts];
  __shared__ float red[kSymThreads / 64][5];
  __shared__ int s_imin[kPts];
  const int R = rows_of(num_rois_dev, R_cap);
  const int sym_items = *nsym * nchunk;
  const int items = sym_items + R;  // then one plain item per row (add_plain_row)
  // nearest indices from k_add_search when its Morton orders exist (else the full scan here)
  const int32_t* nearest = nearest_in && *perm_ok ? nearest_in : nullptr;
  const int grp = threadIdx.x / kSymLanes, lt = threadIdx.x % kSymLanes;
  const int quarter = ((P + kSymGroups - 1) / kSymGroups + kBlk - 1) / kBlk * kBlk;
  const int c0 = grp * quarter, c1 = min(P, c0 + quarter);
  // items are handed out by an atomic counter (zeroed by k_add_prep), so a
  // workgroup that finishes early takes the next (row, chunk)
  __shared__ int s_item;
  for (;;) {
  __syncthreads();
  if (threadIdx.x == 0) s_item = atomicAdd(queue, 1);
  __syncthreads();
  const int item = s_item;
  if (item >= items) break;
  if (item >= sym_items) {  // workgroup-uniform
    add_plain_row(item - sym_items, pred, target, points, symmetry, R, C, P, margin, norm_rows, norm_rows_dev,
                  nchunk, rcls, partial, red);
    continue;  // the loop head synchronises before red is reused
  }
  // full chunks of every symmetric row first, the rows' short last chunks
  // (P % kPts points: cheaper, see the scan below) after them, so the short
  // ones fill the tail of the queue instead of opening a second round of
  // full-cost items
  const int nfull = P / kPts, nsym_rows = *nsym;
  int n, chunk, slot;
  if (item < nsym_rows * nfull) {
    slot = item / nfull;
    chunk = item % nfull;
  } else {
    slot = item - nsym_rows * nfull;
    chunk = nfull;
  }
  n = sym_rows[slot];
  const int PC = 4 * C;
  const int cls = rcls[n];
  float* out = partial + ((size_t)n * nchunk + chunk) * 5;
  const float* tq = target + (size_t)n * PC + 4 * cls;
  const float* pq = pred + (size_t)n * PC + 4 * cls;
  float Rg[9], Rp[9];
  quat2rot(tq[0], tq[1], tq[2], tq[3], Rg);
  const float s = pq[0], u = pq[1], v = pq[2], w = pq[3];
  quat2rot(s, u, v, w, Rp);
  const float* pts = points + (size_t)cls * P * 3;
  if (nearest) {  // the nearest points come from k_add_search (pruned search): no staging, no scan
    for (int jj = threadIdx.x; jj < kPts; jj += blockDim.x) {
      const int p = chunk * kPts + jj;
      s_imin[jj] = p < P ? nearest[(size_t)slot * P + p] : -1;
    }
    __syncthreads();
  } else {
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const float X0 = pts[i * 3 + 0], X1 = pts[i * 3 + 1], X2 = pts[i * 3 + 2];
    gpts[i] = make_float4(Rg[0] * X0 + Rg[1] * X1 + Rg[2] * X2, Rg[3] * X0 + Rg[4] * X1 + Rg[5] * X2,
                          Rg[6] * X0 + Rg[7] * X1 + Rg[8] * X2, 0.f);
  }
  __syncthreads();
  // kPPL query points per lane (points p0 + k*kSymLanes): each broadcast
  // candidate read serves kPPL distances and the lane carries kPPL
  // independent first-minimum chains
  float qx[kPPL], qy[kPPL], qz[kPPL], Xq[kPPL][3];
  int pq_[kPPL];
#pragma unroll
  for (int k = 0; k < kPPL; k++) {
    const int p = chunk * kPts + k * kSymLanes + lt;
    pq_[k] = p;
    const int pp = p < P ? p : 0;
    Xq[k][0] = pts[pp * 3 + 0]; Xq[k][1] = pts[pp * 3 + 1]; Xq[k][2] = pts[pp * 3 + 2];
    qx[k] = Rp[0] * Xq[k][0] + Rp[1] * Xq[k][1] + Rp[2] * Xq[k][2];
    qy[k] = Rp[3] * Xq[k][0] + Rp[4] * Xq[k][1] + Rp[5] * Xq[k][2];
    qz[k] = Rp[6] * Xq[k][0] + Rp[7] * Xq[k][1] + Rp[8] * Xq[k][2];
  }
  // Nearest GT-rotated model point of this group's range [c0, c1) with the
  // reference's first-minimum semantics (strict <, index order, NaN never
  // wins; cu.cc:150-172), in two exact steps: a running minimum over blocks
  // of kBlk candidates (block minimum by v_min3 -- fminf drops NaN like the
  // strict < does; the running minimum updates only on a strictly smaller
  // block minimum, remembering the block), then the first index of that block
  // whose distance, recomputed by the same expression, equals the minimum.
  // The per-candidate compare/select pair of a direct scan becomes ~1/2 min
  // (kBlk 8: one compare + two selects per 8 candidates instead of per 4).
  auto dist_to = [&](int k, const float4& c) {
    return (qx[k] - c.x) * (qx[k] - c.x) + (qy[k] - c.y) * (qy[k] - c.y) + (qz[k] - c.z) * (qz[k] - c.z);
  };
  float dmin[kPPL];
  int iblk[kPPL];
#pragma unroll
  for (int k = 0; k < kPPL; k++) { dmin[k] = FLT_MAX; iblk[k] = -1; }
  // query points in pairs (k, k + 1): every sub / mul / add of a distance is
  // one packed-fp32 instruction over two evaluations, in the scalar
  // expression's association order (bitwise the same as dist_to)
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 px[kPPL / 2], py[kPPL / 2], pz[kPPL / 2];
#pragma unroll
  for (int h = 0; h < kPPL / 2; h++) {
    px[h] = (f2){qx[2 * h], qx[2 * h + 1]};
    py[h] = (f2){qy[2 * h], qy[2 * h + 1]};
    pz[h] = (f2){qz[2 * h], qz[2 * h + 1]};
  }
  // NP query pairs per lane: an item whose queries fit in the first
  // 2 * kSymLanes lanes' slots (a row's short last chunk) scans with one pair
  auto scan = [&](auto np_c) {
    constexpr int NP = decltype(np_c)::value;
    int i = c0;
    for (; i + kBlk <= c1; i += kBlk) {
      float4 c[kBlk];
#pragma unroll
      for (int j = 0; j < kBlk; j++) c[j] = gpts[i + j];
#pragma unroll
      for (int h = 0; h < NP; h++) {
        f2 d[kBlk];
#pragma unroll
        for (int j = 0; j < kBlk; j++) {
          const f2 ex = px[h] - c[j].x, ey = py[h] - c[j].y, ez = pz[h] - c[j].z;
          d[j] = ex * ex + ey * ey + ez * ez;
        }
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int k = 2 * h + e;
          float bm = fminf(d[0][e], d[1][e]);  // min3 chains: (kBlk - 1) / 2 instructions
#pragma unroll
          for (int j = 2; j < kBlk; j += 2) bm = fminf(bm, fminf(d[j][e], d[j + 1][e]));
          if (bm < dmin[k]) { dmin[k] = bm; iblk[k] = i; }
        }
      }
    }
    for (; i < c1; i++) {  // ragged tail: blocks of one
      const float4 c = gpts[i];
#pragma unroll
      for (int k = 0; k < 2 * NP; k++) {
        const float d = dist_to(k, c);
        if (d < dmin[k]) { dmin[k] = d; iblk[k] = i; }
      }
    }
  };
  const int nq = min(kPts, P - chunk * kPts);  // query points of this item
  if (nq > 2 * kSymLanes) scan(std::integral_constant<int, kPPL / 2>{});
  else scan(std::integral_constant<int, 1>{});
  if (grp > 0) {
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
      mdist[grp - 1][k * kSymLanes + lt] = dmin[k];
      midx[grp - 1][k * kSymLanes + lt] = iblk[k];
    }
  }
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
#pragma unroll
      for (int g = 0; g < kSymGroups - 1; g++) {  // group order, strict <: the earliest range wins ties
        const float d = mdist[g][k * kSymLanes + lt];
        if (d < dmin[k]) { dmin[k] = d; iblk[k] = midx[g][k * kSymLanes + lt]; }
      }
      int im = -1;
      if (iblk[k] >= 0) {
        const int e = min(iblk[k] + kBlk, P);
        for (int j = iblk[k]; j < e; j++)
          if (dist_to(k, gpts[j]) == dmin[k]) { im = j; break; }
      }
      s_imin[k * kSymLanes + lt] = im;
    }
  }
  __syncthreads();
  }  // full scan
  // per-point loss and gradient terms (cu.cc:174-203), one point per thread
  // over the whole workgroup
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int jj = threadIdx.x; jj < kPts; jj += blockDim.x) {
    const int p = chunk * kPts + jj;
    if (p >= P) continue;
    const int im = s_imin[jj] < 0 ? p : s_imin[jj];  // no finite distance (index_min unset in the reference)
    const float X0 = pts[p * 3 + 0], X1 = pts[p * 3 + 1], X2 = pts[p * 3 + 2];
    const float x1 = Rp[0] * X0 + Rp[1] * X1 + Rp[2] * X2;  // = the scan's query point, same expression
    const float y1 = Rp[3] * X0 + Rp[4] * X1 + Rp[5] * X2;
    const float z1 = Rp[6] * X0 + Rp[7] * X1 + Rp[8] * X2;
    float x2, y2, z2;
    if (nearest) {  // the GT-rotated point by the staging's expression (the same bits as gpts[im])
      const float Y0 = pts[im * 3 + 0], Y1 = pts[im * 3 + 1], Y2 = pts[im * 3 + 2];
      x2 = Rg[0] * Y0 + Rg[1] * Y1 + Rg[2] * Y2;
      y2 = Rg[3] * Y0 + Rg[4] * Y1 + Rg[5] * Y2;
      z2 = Rg[6] * Y0 + Rg[7] * Y1 + Rg[8] * Y2;
    } else {
      const float4 cm = gpts[im];
      x2 = cm.x, y2 = cm.y, z2 = cm.z;
    }
    const int Rn = norm_rows_dev ? *norm_rows_dev : (norm_rows > 0 ? norm_rows : R);
    const float bn = (float)(Rn * P), rbn = 1.f / bn;
    const double ln = 2.0 * (double)Rn * (double)P, rln = 1.0 / ln;
    const float dist = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2);
    if (!(dist < margin)) {  // cu.cc:178-179
      acc[0] += (float)div_rn((double)(dist - margin), ln, rln);  // cu.cc:181
      // derivative matrices of Rp w.r.t. (s, u, v, w) (cu.cc:97-139)
      const float d0[9] = {2 * s, -2 * w, 2 * v, 2 * w, 2 * s, -2 * u, -2 * v, 2 * u, 2 * s};
      const float d1[9] = {2 * u, 2 * v, 2 * w, 2 * v, -2 * u, -2 * s, 2 * w, 2 * s, -2 * u};
      const float d2[9] = {-2 * v, 2 * u, 2 * s, 2 * u, 2 * v, 2 * w, -2 * s, 2 * w, -2 * v};
      const float d3[9] = {-2 * w, -2 * s, 2 * u, 2 * s, -2 * w, 2 * v, 2 * u, 2 * v, 2 * w};
      const float X[3] = {X0, X1, X2};
      const float df[3] = {x1 - x2, y1 - y2, z1 - z2};
      float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;  // this point's terms, reference order
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 3; b++) {  // cu.cc:183-203, same operation order
          e0 += div_rn(df[a] * X[b] * d0[a * 3 + b], bn, rbn);
          e1 += div_rn(df[a] * X[b] * d1[a * 3 + b], bn, rbn);
          e2 += div_rn(df[a] * X[b] * d2[a * 3 + b], bn, rbn);
          e3 += div_rn(df[a] * X[b] * d3[a * 3 + b], bn, rbn);
        }
      acc[1] += e0; acc[2] += e1; acc[3] += e2; acc[4] += e3;
    }
  }
#pragma unroll
  for (int q = 0; q < 5; q++) acc[q] = pcnn::wave_sum(acc[q]);
  if (pcnn::lane_id() == 0)
    for (int q = 0; q < 5; q++) red[threadIdx.x >> 6][q] = acc[q];
  __syncthreads();
  if (threadIdx.x < 5) {  // fixed order over the waves
    float t = 0.f;
    for (int i = 0; i < kSymThreads / 64; i++) t += red[i][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();  // red / gpts / mdist reused by the next item
  }
}

// ---------------------------------------------------------------------------
// Pruned ADD-S nearest-point search (symmetric rows).  The reference scans
// all P GT-rotated model points for each of the P predicted points
// (cu.cc:150-172: O(P^2) per row, the loss's whole cost).  Rotations keep
// distances, so the model's points are grouped ONCE per call, in model space:
// a Morton order per symmetric class (k_add_order, beside the row
// classification), blocks of kPrBlk consecutive points and super-blocks of
// kPrSup blocks.  Per row the blocks' bounding spheres are taken in the
// rotated frame (centre = mean, radius = the largest point distance, padded);
// each lane owns one query point (queries in the same Morton order, so a
// wave's 64 queries are close together), seeds its minimum with the block
// nearest it, then visits the blocks and skips -- wave-uniformly -- every
// super-block / block whose sphere lies farther than the current minimum
// from all 64 queries.  Candidates that are
// visited get the reference's exact fp32 distance expression and the
// first-minimum rule (lowest point index among equal minima, NaN never
// wins), so the result is the full scan's index bit for bit; the bounds
// carry 1e-4 relative + 1e-18 absolute slack (far above fp32 rounding), and a
// non-finite sphere is never skipped.
constexpr int kPrBlk = 8;       // candidates per block
constexpr int kPrSup = 8;       // blocks per super-block
constexpr int kPrThreads = 512;  // queries per search item (one per lane, 8 waves)
constexpr int kPrMaxP = 4096;   // Morton sort of <= 4096 keys in LDS
#ifndef ADD_PR_GRID
#define ADD_PR_GRID 768
#endif

__device__ __forceinline__ float fl_dist(float ax, float ay, float az, float bx, float by, float bz) {
  return (ax - bx) * (ax - bx) + (ay - by) * (ay - by) + (az - bz) * (az - bz);  // dist_to's expression
}

// Morton order of each symmetric class's model points (10 bits per axis of
// the class's bounding box; ties by index): perm[c][i] = the i-th point.
__global__ void __launch_bounds__(1024) k_add_order(const float* __restrict__ points,
                                                     const float* __restrict__ symmetry, int P,
                                                     int32_t* __restrict__ perm) {
  __shared__ unsigned long long key[kPrMaxP];
  __shared__ float red[6][16];
  const int c = blockIdx.x, t = threadIdx.x;
  if (!(symmetry[c] > 0)) return;
  const float* pts = points + (size_t)c * P * 3;
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = t; i < P; i += blockDim.x)
    for (int a = 0; a < 3; a++) {
      lo[a] = fminf(lo[a], pts[i * 3 + a]);
      hi[a] = fmaxf(hi[a], pts[i * 3 + a]);
    }
  for (int a = 0; a < 3; a++) {
    for (int o = 32; o > 0; o >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], o));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], o));
    }
    if (pcnn::lane_id() == 0) {
      red[a][t >> 6] = lo[a];
      red[3 + a][t >> 6] = hi[a];
    }
  }
  __syncthreads();
  for (int a = 0; a < 3; a++) {
    lo[a] = red[a][0];
    hi[a] = red[3 + a][0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
      lo[a] = fminf(lo[a], red[a][w]);
      hi[a] = fmaxf(hi[a], red[3 + a][w]);
    }
  }
  int n2 = 1;
  while (n2 < P) n2 <<= 1;
  for (int i = t; i < n2; i += blockDim.x) {
    unsigned long long k = ~0ull;
    if (i < P) {
      unsigned code = 0;
      unsigned q[3];
      for (int a = 0; a < 3; a++) {
        const float ext = hi[a] - lo[a];
        const float f = ext > 0.f ? (pts[i * 3 + a] - lo[a]) / ext * 1023.f : 0.f;
        q[a] = f > 0.f ? (f < 1023.f ? (unsigned)f : 1023u) : 0u;  // NaN -> 0
      }
      for (int b = 0; b < 10; b++)
        for (int a = 0; a < 3; a++) code |= ((q[a] >> b) & 1u) << (3 * b + a);
      k = ((unsigned long long)code << 13) | (unsigned)i;
    }
    key[i] = k;
  }
  __syncthreads();
  for (int k = 2; k <= n2; k <<= 1)  // bitonic sort, ascending
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < n2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = key[i], b = key[l];
          const bool up = (i & k) == 0;
          if (up ? a > b : a < b) {
            key[i] = b;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = t; i < P; i += blockDim.x) perm[(size_t)c * P + i] = (int32_t)(key[i] & 0x1FFFull);
}

// The search: item = (symmetric row, kPrThreads queries of its Morton order);
// nearest[slot][p] = the index of point p's nearest GT-rotated model point
// (first minimum), -1 when no distance is finite (the reference leaves
// index_min unset; the loss then uses p itself).
__global__ void __launch_bounds__(kPrThreads) k_add_search(const float* __restrict__ pred,
                                                           const float* __restrict__ target,
                                                           const float* __restrict__ points, int C, int P,
                                                           const int32_t* __restrict__ rcls,
                                                           const int32_t* __restrict__ sym_rows,
                                                           const int32_t* __restrict__ nsym,
                                                           const int32_t* __restrict__ perm,
                                                           const int32_t* __restrict__ perm_ok,
                                                           int32_t* __restrict__ queue,
                                                           int32_t* __restrict__ nearest,
                                                           int32_t* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float4 plds[];
  const int nb = (P + kPrBlk - 1) / kPrBlk, nsb = (nb + kPrSup - 1) / kPrSup;
  float4* gp = plds;        // [P] GT-rotated points in Morton order, w = the point's index (int bits)
  float4* blk = gp + P;     // [nb] block spheres (centre, radius)
  float4* sup = blk + nb;   // [nsb] super-block spheres
  __shared__ int s_item;
  const int nqi = (P + kPrThreads - 1) / kPrThreads;
  const int items = *perm_ok ? *nsym * nqi : 0;  // no Morton orders: k_add_rows scans in full
  const int t = threadIdx.x;
  for (;;) {
    __syncthreads();
    if (t == 0) s_item = atomicAdd(queue, 1);
    __syncthreads();
    const int item = s_item;
    if (item >= items) break;
    const int slot = item / nqi, qi = item % nqi;
    const int n = sym_rows[slot];
    const int cls = rcls[n];
    const int PC = 4 * C;
    const float* tq = target + (size_t)n * PC + 4 * cls;
    const float* pq = pred + (size_t)n * PC + 4 * cls;
    float Rg[9], Rp[9];
    quat2rot(tq[0], tq[1], tq[2], tq[3], Rg);
    quat2rot(pq[0], pq[1], pq[2], pq[3], Rp);
    const float* pts = points + (size_t)cls * P * 3;
    const int32_t* pm = perm + (size_t)cls * P;
#pragma unroll 4
    for (int i = t; i < P; i += kPrThreads) {
      const int j = pm[i];
      const float X0 = pts[j * 3 + 0], X1 = pts[j * 3 + 1], X2 = pts[j * 3 + 2];
      gp[i] = make_float4(Rg[0] * X0 + Rg[1] * X1 + Rg[2] * X2, Rg[3] * X0 + Rg[4] * X1 + Rg[5] * X2,
                          Rg[6] * X0 + Rg[7] * X1 + Rg[8] * X2, __int_as_float(j));
    }
    __syncthreads();
    for (int b = t; b < nb; b += blockDim.x) {  // block spheres
      const int j0 = b * kPrBlk, j1 = min(j0 + kPrBlk, P);
      float sx = 0.f, sy = 0.f, sz = 0.f;
      for (int j = j0; j < j1; j++) {
        sx += gp[j].x;
        sy += gp[j].y;
        sz += gp[j].z;
      }
      const float inv = 1.f / (float)(j1 - j0);
      const float mx = sx * inv, my = sy * inv, mz = sz * inv;
      float r = INFINITY;  // a non-finite point (or an overflowing sum): never skipped
      if (isfinite(mx) && isfinite(my) && isfinite(mz)) {
        float r2 = 0.f;
        for (int j = j0; j < j1; j++) r2 = fmaxf(r2, fl_dist(gp[j].x, gp[j].y, gp[j].z, mx, my, mz));
        if (isfinite(r2)) r = sqrtf(r2) * 1.0001f + 1e-18f;
      }
      blk[b] = make_float4(mx, my, mz, r);
    }
    __syncthreads();
    for (int sb = t; sb < nsb; sb += blockDim.x) {  // super-block spheres over the blocks' spheres
      const int b0 = sb * kPrSup, b1 = min(b0 + kPrSup, nb);
      float sx = 0.f, sy = 0.f, sz = 0.f;
      for (int b = b0; b < b1; b++) {
        sx += blk[b].x;
        sy += blk[b].y;
        sz += blk[b].z;
      }
      const float inv = 1.f / (float)(b1 - b0);
      const float mx = sx * inv, my = sy * inv, mz = sz * inv;
      float r = 0.f;
      for (int b = b0; b < b1; b++)
        r = fmaxf(r, sqrtf(fl_dist(blk[b].x, blk[b].y, blk[b].z, mx, my, mz)) * 1.0001f + blk[b].w);
      if (!(isfinite(mx) && isfinite(my) && isfinite(mz) && isfinite(r))) r = INFINITY;
      for (int b = b0; b < b1; b++)
        if (!(blk[b].w < INFINITY)) r = INFINITY;  // (fmaxf would drop a NaN radius)
      sup[sb] = make_float4(mx, my, mz, r + 1e-18f);
    }
    __syncthreads();
    const int qpos = qi * kPrThreads + t;
    const bool valid = qpos < P;
    if (__ballot(valid) == 0ull) continue;  // a wave with no query of this item (the loop head syncs)
    const int p = pm[valid ? qpos : 0];
    const float X0 = pts[p * 3 + 0], X1 = pts[p * 3 + 1], X2 = pts[p * 3 + 2];
    const float qx = Rp[0] * X0 + Rp[1] * X1 + Rp[2] * X2;  // k_add_rows' query expression
    const float qy = Rp[3] * X0 + Rp[4] * X1 + Rp[5] * X2;
    const float qz = Rp[6] * X0 + Rp[7] * X1 + Rp[8] * X2;
    float dmin = FLT_MAX;  // k_add_rows' start value: strict <, so a distance of FLT_MAX never wins
    int best = -1;         // the model index of the nearest point so far
    // exact distances to block b's points, first-minimum update (lowest model
    // index among equal minima: the blocks arrive out of index order)
    auto scan_block = [&](int b) {
      const int j0 = b * kPrBlk;
      float4 c[kPrBlk];
      float d[kPrBlk];
#pragma unroll
      for (int e = 0; e < kPrBlk; e++) {
        c[e] = gp[min(j0 + e, P - 1)];
        d[e] = j0 + e < P ? fl_dist(qx, qy, qz, c[e].x, c[e].y, c[e].z) : INFINITY;
      }
      float bm = fminf(d[0], d[1]);  // NaN never wins (fminf drops it, the strict < below too)
#pragma unroll
      for (int e = 2; e < kPrBlk; e += 2) bm = fminf(bm, fminf(d[e], d[e + 1]));
      if (bm < dmin || (bm == dmin && best >= 0)) {
        int bi = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < kPrBlk; e++) {
          const int j = __float_as_int(c[e].w);
          if (d[e] == bm && j < bi) bi = j;
        }
        if (bm < dmin) {
          dmin = bm;
          best = bi;
        } else if (bi < best) {
          best = bi;
        }
      }
    };
    // seed: the block nearest the query (by centre) inside the super-block
    // nearest the query, scanned exactly -- dmin starts near its final value
    {
      float bd = INFINITY;
      int bsel = 0;
      for (int sb = 0; sb < nsb; sb++) {
        const float4 m = sup[sb];
        const float d2 = fl_dist(qx, qy, qz, m.x, m.y, m.z);
        if (d2 < bd) {
          bd = d2;
          bsel = sb;
        }
      }
      bd = INFINITY;
      int b0 = bsel * kPrSup, bpick = b0;
      for (int b = b0; b < min(b0 + kPrSup, nb); b++) {  // per-lane reads (each lane its own super-block)
        const float4 m = blk[b];
        const float d2 = fl_dist(qx, qy, qz, m.x, m.y, m.z);
        if (d2 < bd) {
          bd = d2;
          bpick = b;
        }
      }
      if (valid) scan_block(bpick);
    }
    // s = sqrt(dmin) padded: a sphere (centre at fl_dist d2, radius r) can
    // hold no point at a distance <= dmin when d2 (1 - 3e-4) > ((r + s +
    // 1e-18)^2 (1 + 1e-4)) -- sqrt-free, with slack far above fp32 rounding;
    // an infinite radius or s (no finite distance yet) and a NaN never skip
    float dlast = dmin, s_ = sqrtf(dmin) * 1.0001f;
    int nscan = 0;
    auto far_from = [&](const float4& m) {
#ifdef ADD_PR_NOPRUNE  // timing ablation: visit every block
      return m.w < -1.f;
#endif
      const float d2 = fl_dist(qx, qy, qz, m.x, m.y, m.z);
      const float rr = m.w + s_ + 1e-18f;
      return d2 * 0.9997f > rr * rr * 1.0001f;
    };
#ifdef ADD_PR_STAGE_ONLY  // timing ablation (wrong results): staging and seeding only
    if (valid) nearest[(size_t)slot * P + p] = best;
    continue;
#endif
    for (int sb = 0; sb < nsb; sb++) {
      if (dmin != dlast) {
        dlast = dmin;
        s_ = sqrtf(dmin) * 1.0001f;
      }
      if (__ballot(valid && !far_from(sup[sb])) == 0ull) continue;
      const int b1 = min(sb * kPrSup + kPrSup, nb);
      for (int b = sb * kPrSup; b < b1; b++) {
        if (dmin != dlast) {
          dlast = dmin;
          s_ = sqrtf(dmin) * 1.0001f;
        }
        if (__ballot(valid && !far_from(blk[b])) == 0ull) continue;
        scan_block(b);
        nscan++;
      }
    }
    if (pcnn::lane_id() == 0) {  // per wave: blocks scanned of the blocks held (a no-op for the result)
      atomicAdd(stats, nscan);
      atomicAdd(stats + 1, nb);
    }
    if (valid) nearest[(size_t)slot * P + p] = best;
  }
}

// Row classes once (first class with weight > 0, cu.cc:47-52) and the
// ascending list of symmetric rows (ballot scan, one workgroup: deterministic).
__global__ void __launch_bounds__(1024) k_add_prep(const float* __restrict__ weight, const float* __restrict__ symmetry,
                                                    int R_cap, const int32_t* __restrict__ num_rois_dev, int C,
                                                    int32_t* __restrict__ rcls, int32_t* __restrict__ sym_rows,
                                                    int32_t* __restrict__ nsym, int32_t* __restrict__ queue,
                                                    int32_t* __restrict__ squeue, int32_t* __restrict__ perm_ok,
                                                    int order, int32_t* __restrict__ stats) {
  __shared__ int wcount[16];
  __shared__ int base;
  const int R = rows_of(num_rois_dev, R_cap);
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int n0 = 0; n0 < R; n0 += blockDim.x) {
    const int n = n0 + threadIdx.x;
    int cls = -1;
    if (n < R) {
      cls = row_class(weight, n, C);
      rcls[n] = cls;
    }
    const bool sym = n < R && cls >= 0 && symmetry[cls] > 0;
    const uint64_t m = __ballot(sym);
    if (lane == 0) wcount[wave] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; w++) off += wcount[w];
    if (sym) sym_rows[off + __popcll(m & pcnn::lanemask_lt())] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += wcount[w];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *nsym = base;
    *queue = 0;
    *squeue = 0;
    *perm_ok = order;
    stats[0] = stats[1] = 0;
  }
}

__device__ __forceinline__ void finish_row(int n, int R, int C, int nchunk, const int32_t* __restrict__ rcls,
                                           const float* __restrict__ partial, float* __restrict__ row_loss,
                                           float* __restrict__ bottom_diff, int lane) {
  if (n >= R) return;
  const int cls = rcls[n];
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = lane; k < nchunk; k += 64)
    for (int q = 0; q < 5; q++) s[q] += partial[((size_t)n * nchunk + k) * 5 + q];
#pragma unroll
  for (int q = 0; q < 5; q++) s[q] = pcnn::wave_sum(s[q]);
  const int PC = 4 * C;
  for (int col = lane; col < PC; col += 64) {
    float vv = 0.f;
    if (cls >= 0 && col >= 4 * cls && col < 4 * cls + 4) vv = s[1 + col - 4 * cls];
    bottom_diff[(size_t)n * PC + col] = vv;
  }
  if (lane == 0) row_loss[n] = cls >= 0 ? s[0] : 0.f;
}

// One wave per row: fold the chunk partials (fixed tree), write the row of
// bottom_diff (zeros except the class's 4 channels) and the row loss.
// Measured and dropped: the scalar total added by the last workgroup to
// finish (device-scope counter): the agent-scope release fence of each of the
// 288 workgroups writes back the XCD's L2, 12 -> 25 us for the pair of launches.
__global__ void __launch_bounds__(256) k_add_finish_rows(int R_cap, const int32_t* __restrict__ num_rois_dev, int C,
                                                          int nchunk, const int32_t* __restrict__ rcls,
                                                          const float* __restrict__ partial,
                                                          float* __restrict__ row_loss,
                                                          float* __restrict__ bottom_diff) {
  const int R = rows_of(num_rois_dev, R_cap);
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  finish_row(n, R, C, nchunk, rcls, partial, row_loss, bottom_diff, pcnn::lane_id());
}

// k_add_finish_rows + the pose head's backward in one pass (the step's fused
// tail, pcnn_add_loss_fwd_head_bwd): the row's four gradient sums go straight
// into d pred (times the ADD gradient op's top_diff[0], cu.cc:346-354) and on
// through tanh * poses_weight -> l2_normalize (pose_head.hip k_head_bwd, the
// same helper), so the d_pred row is never re-read.  4 C <= 256.
__global__ void __launch_bounds__(256) k_add_finish_head(int R_cap, const int32_t* __restrict__ num_rois_dev, int C,
                                                          int nchunk, const int32_t* __restrict__ rcls,
                                                          const float* __restrict__ partial,
                                                          float* __restrict__ row_loss,
                                                          float* __restrict__ bottom_diff,
                                                          const float* __restrict__ t_in,
                                                          const float* __restrict__ pw,
                                                          const float* __restrict__ pred,
                                                          const float* __restrict__ dscale, float* __restrict__ dy8) {
  const int R = rows_of(num_rois_dev, R_cap);
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = pcnn::lane_id();
  if (n >= R) return;
  const int cls = rcls[n];
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = lane; k < nchunk; k += 64)
    for (int q = 0; q < 5; q++) s[q] += partial[((size_t)n * nchunk + k) * 5 + q];
#pragma unroll
  for (int q = 0; q < 5; q++) s[q] = pcnn::wave_sum(s[q]);
  const int PC = 4 * C;
  const float g = dscale ? dscale[0] : 1.f;
  float dp[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int col = lane + 64 * k;
    float vv = 0.f;
    if (cls >= 0 && col >= 4 * cls && col < 4 * cls + 4) vv = s[1 + col - 4 * cls];
    if (col < PC) bottom_diff[(size_t)n * PC + col] = vv;
    dp[k] = col < PC ? g * vv : 0.f;
  }
  if (lane == 0) row_loss[n] = cls >= 0 ? s[0] : 0.f;
  pcnn_head::head_bwd_row(dp, t_in, pw, pred, n, PC, lane, dy8);
}

// Scalar loss: fixed-order sum of the row losses (thrust::reduce, cu.cc:333-334).
__global__ void __launch_bounds__(1024) k_add_total(int R_cap, const int32_t* __restrict__ num_rois_dev,
                                                     const float* __restrict__ row_loss, float* __restrict__ loss) {
  __shared__ float red[16];
  const int R = rows_of(num_rois_dev, R_cap);
  float my = 0.f;
  for (int n = threadIdx.x; n < R; n += blockDim.x) my += row_loss[n];
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

extern "C" int pcnn_div_rn_check(const float* x, float b, int n, int dbl, float* out, void* stream) {
  PCNN_REQUIRE(x && out && n >= 0 && b != 0.f);
  if (n == 0) return PCNN_OK;
  hipLaunchKernelGGL(k_div_rn_check, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, b, n, dbl, out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

// The loss's workspace, carved the same way by every entry point.  The
// pruned search's Morton orders (C x P) and nearest indices (R_cap x P) are
// there whenever P <= kPrMaxP.
struct AddWs {
  float* partial;
  int32_t *rcls, *sym_rows, *nsym, *queue, *squeue;
  float* row_loss;
  int32_t *perm, *nearest;
  int32_t* perm_ok;  // device flag: the Morton orders were built by this call's prep
  int32_t* stats;    // the search's [blocks scanned, blocks held] over the call's queries (diagnostics)
};
static AddWs add_carve(void* workspace, int R_cap, int C, int P, size_t* bytes) {
  const int nchunk = (P + kPts - 1) / kPts;
  const size_t R = (size_t)(R_cap > 0 ? R_cap : 1);
  pcnn::Carve cv(workspace);
  AddWs w;
  w.partial = cv.take<float>(R * nchunk * 5);
  w.rcls = cv.take<int32_t>(R);
  w.sym_rows = cv.take<int32_t>(R);
  w.nsym = cv.take<int32_t>(1);
  w.queue = cv.take<int32_t>(1);
  w.row_loss = cv.take<float>(R);
  w.squeue = cv.take<int32_t>(1);
  w.perm_ok = cv.take<int32_t>(1);
  w.stats = cv.take<int32_t>(2);
  const bool pr = P <= kPrMaxP;
  w.perm = pr ? cv.take<int32_t>((size_t)(C > 0 ? C : 1) * P) : nullptr;
  w.nearest = pr ? cv.take<int32_t>(R * P) : nullptr;
  if (bytes) *bytes = cv.off + 256;
  return w;
}

// Which nearest-point search the symmetric rows use: the full O(P^2) scan
// (the default) or the pruned one (PCNN_ADD_SEARCH=pruned, P <= kPrMaxP; the
// same bits).  Measured on the bench's rows (round 6, scripts/add_bench.py):
// the pruned search visits 16 % of the blocks (13 % for near-correct
// predictions) but its per-block sphere tests are a latency-bound chain of
// LDS read -> distance -> ballot -> branch, so the op runs 314 us against the
// full scan's 212 us (and 132 us with the search ablated): not the default.
static bool add_pruned(int P) {
  if (P > kPrMaxP) return false;
  const char* e = getenv("PCNN_ADD_SEARCH");
  return e && strcmp(e, "pruned") == 0;
}

// Byte offsets inside the workspace of the search's diagnostics (tests and
// benches): what = 0 the Morton orders (C x P int32), 1 the [scanned, held]
// block counters of the last search.  -1 when the pruned search is off (P > kPrMaxP).
extern "C" long pcnn_add_loss_ws_offset(int R_cap, int C, int P, int what) {
  char* const base = (char*)(uintptr_t)4096;  // any aligned non-null base: only the offsets are used
  const AddWs w = add_carve(base, R_cap, C, P, nullptr);
  const int32_t* q = what == 0 ? w.perm : what == 1 ? w.stats : nullptr;
  if (!q || !w.perm) return -1;
  return (long)((const char*)q - base);
}

extern "C" size_t pcnn_add_loss_workspace_size(int R_cap, int C, int P) {
  size_t b = 0;
  (void)add_carve(nullptr, R_cap, C, P, &b);
  return b;
}

// the row classification, and the symmetric classes' Morton orders (pruned search)
static void add_launch_prep(const AddWs& w, const float* weight, const float* symmetry, const float* points,
                            int R_cap, const int32_t* num_rois_dev, int C, int P, hipStream_t st) {
  const int order = w.perm && points && add_pruned(P) ? 1 : 0;
  hipLaunchKernelGGL(k_add_prep, dim3(1), dim3(1024), 0, st, weight, symmetry, R_cap, num_rois_dev, C, w.rcls,
                     w.sym_rows, w.nsym, w.queue, w.squeue, w.perm_ok, order, w.stats);
  if (order) hipLaunchKernelGGL(k_add_order, dim3(C), dim3(1024), 0, st, points, symmetry, P, w.perm);
}

// the per-point sums: the symmetric rows' pruned nearest-point search first
// (when selected), then the persistent (row, chunk) queue of k_add_rows
static int add_launch_rows(const AddWs& w, const float* pred, const float* target, const float* weight,
                           const float* points, const float* symmetry, int R_cap, const int32_t* num_rois_dev,
                           int C, int P, float margin, int loss_norm_rows, const int32_t* loss_norm_rows_dev,
                           hipStream_t st) {
  const int nchunk = (P + kPts - 1) / kPts;
  const bool pr = add_pruned(P);
  if (pr) {
    const int nb = (P + kPrBlk - 1) / kPrBlk, nsb = (nb + kPrSup - 1) / kPrSup;
    const size_t lds = (size_t)(P + nb + nsb) * sizeof(float4);
    if (lds > 64 * 1024 && hipFuncSetAttribute((const void*)k_add_search, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) != hipSuccess)
      return PCNN_EHIP;
    const long items = (long)R_cap * ((P + kPrThreads - 1) / kPrThreads);
    const int grid = (int)(items < ADD_PR_GRID ? items : ADD_PR_GRID);
    hipLaunchKernelGGL(k_add_search, dim3(grid), dim3(kPrThreads), lds, st, pred, target, points, C, P, w.rcls,
                       w.sym_rows, w.nsym, w.perm, w.perm_ok, w.squeue, w.nearest, w.stats);
  }
  // one persistent grid: symmetric (row, chunk) items of the device-side list, then the plain rows
  const long sym_items = (long)R_cap * nchunk + R_cap;
  const int sym_grid = (int)(sym_items < ADD_GRID ? sym_items : ADD_GRID);
  // (dynamic LDS for the full scan's staging either way: a prep without the
  // points leaves perm_ok 0 and k_add_rows then scans)
  hipLaunchKernelGGL(k_add_rows, dim3(sym_grid), dim3(kSymThreads), (size_t)P * sizeof(float4), st, pred,
                     target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin, loss_norm_rows,
                     loss_norm_rows_dev, nchunk, w.rcls, w.sym_rows, w.nsym, w.queue, w.partial,
                     pr ? w.nearest : nullptr, w.perm_ok);
  return PCNN_OK;
}

static int add_loss_fwd(const float* pred, const float* target, const float* weight, const float* points,
                        const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P, float margin,
                        int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss, float* bottom_diff,
                        void* workspace, size_t workspace_bytes, bool prepared, void* stream) {
  PCNN_REQUIRE(pred && target && weight && points && symmetry && loss && bottom_diff && workspace);
  PCNN_REQUIRE(R_cap > 0 && C > 0 && P > 0 && P <= kMaxPointsLds);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = (P + kPts - 1) / kPts;
  const AddWs w = add_carve(workspace, R_cap, C, P, nullptr);
  if (!prepared) add_launch_prep(w, weight, symmetry, points, R_cap, num_rois_dev, C, P, st);
  const int rc = add_launch_rows(w, pred, target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin,
                                 loss_norm_rows, loss_norm_rows_dev, st);
  if (rc != PCNN_OK) return rc;
  hipLaunchKernelGGL(k_add_finish_rows, dim3((R_cap + 3) / 4), dim3(256), 0, st, R_cap, num_rois_dev, C, nchunk,
                     w.rcls, w.partial, w.row_loss, bottom_diff);
  hipLaunchKernelGGL(k_add_total, dim3(1), dim3(1024), 0, st, R_cap, num_rois_dev, w.row_loss, loss);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_add_loss_fwd(const float* pred, const float* target, const float* weight, const float* points,
                                 const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P,
                                 float margin, int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss,
                                 float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
  return add_loss_fwd(pred, target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin, loss_norm_rows,
                      loss_norm_rows_dev, loss, bottom_diff, workspace, workspace_bytes, false, stream);
}

extern "C" int pcnn_add_loss_prep_points(const float* weight, const float* symmetry, const float* points, int R_cap,
                                         const int32_t* num_rois_dev, int C, int P, void* workspace,
                                         size_t workspace_bytes, void* stream);

// The row classification of pcnn_add_loss_fwd on its own: it reads only the
// weights (the Hough op's targets) and the model points, so a caller can run
// it as soon as they exist, on another stream, off the chain that produces
// the predictions.
extern "C" int pcnn_add_loss_prep(const float* weight, const float* symmetry, int R_cap, const int32_t* num_rois_dev,
                                  int C, int P, void* workspace, size_t workspace_bytes, void* stream) {
  return pcnn_add_loss_prep_points(weight, symmetry, nullptr, R_cap, num_rois_dev, C, P, workspace, workspace_bytes,
                                   stream);
}

// ... with the model points: the symmetric classes' Morton orders for the
// pruned search are built here too (without the points, the prepared loss
// uses the full scan).
extern "C" int pcnn_add_loss_prep_points(const float* weight, const float* symmetry, const float* points, int R_cap,
                                         const int32_t* num_rois_dev, int C, int P, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(weight && symmetry && workspace && R_cap > 0 && C > 0 && P > 0 && P <= kMaxPointsLds);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  const AddWs w = add_carve(workspace, R_cap, C, P, nullptr);
  add_launch_prep(w, weight, symmetry, points, R_cap, num_rois_dev, C, P, (hipStream_t)stream);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_add_loss_fwd_prepared(const float* pred, const float* target, const float* weight,
                                          const float* points, const float* symmetry, int R_cap,
                                          const int32_t* num_rois_dev, int C, int P, float margin,
                                          int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss,
                                          float* bottom_diff, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  return add_loss_fwd(pred, target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin, loss_norm_rows,
                      loss_norm_rows_dev, loss, bottom_diff, workspace, workspace_bytes, true, stream);
}

// The loss with the step's backward tail fused in (prepared rows only): the
// per-point sums (k_add_rows), then one pass that finishes each row's
// bottom_diff and runs the pose head's backward on it into d_y8
// (pcnn_pose_head_bwd with d_pred = bottom_diff, d_pred_scale the ADD
// gradient op's top_diff[0]: the same bits as the two separate launches).
// The scalar loss is left to pcnn_add_loss_total on the same workspace --
// nothing on the backward chain reads it, so a caller can run it on another
// stream after this call.  4 C <= 256.
extern "C" int pcnn_add_loss_fwd_head_bwd(const float* pred, const float* target, const float* weight,
                                          const float* points, const float* symmetry, int R_cap,
                                          const int32_t* num_rois_dev, int C, int P, float margin,
                                          int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* bottom_diff,
                                          void* workspace, size_t workspace_bytes, const float* tanh_out,
                                          const float* d_pred_scale, float* d_y8, void* stream) {
  PCNN_REQUIRE(pred && target && weight && points && symmetry && bottom_diff && workspace && tanh_out && d_y8);
  PCNN_REQUIRE(R_cap > 0 && C > 0 && 4 * C <= 256 && P > 0 && P <= kMaxPointsLds);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = (P + kPts - 1) / kPts;
  const AddWs w = add_carve(workspace, R_cap, C, P, nullptr);
  const int rc = add_launch_rows(w, pred, target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin,
                                 loss_norm_rows, loss_norm_rows_dev, st);
  if (rc != PCNN_OK) return rc;
  pcnn::launch_last(k_add_finish_head, dim3((R_cap + 3) / 4), dim3(256), 0, st, R_cap, num_rois_dev, C, nchunk,
                     w.rcls, w.partial, w.row_loss, bottom_diff, tanh_out, weight, pred, d_pred_scale, d_y8);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

// The scalar loss of a pcnn_add_loss_fwd_head_bwd call (the row losses it left
// in the workspace, summed in the fixed order of pcnn_add_loss_fwd).
extern "C" int pcnn_add_loss_total(int R_cap, const int32_t* num_rois_dev, int C, int P, const void* workspace,
                                   size_t workspace_bytes, float* loss, void* stream) {
  PCNN_REQUIRE(workspace && loss && R_cap > 0 && C > 0 && P > 0);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  const AddWs w = add_carve(const_cast<void*>(workspace), R_cap, C, P, nullptr);
  hipLaunchKernelGGL(k_add_total, dim3(1), dim3(1024), 0, (hipStream_t)stream, R_cap, num_rois_dev, w.row_loss,
                     loss);
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
