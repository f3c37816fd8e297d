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
#include <cfloat>
#include <type_traits>

namespace {

#ifndef ADD_LANES
#define ADD_LANES 64
#endif
constexpr int kSymLanes = ADD_LANES;           // symmetric rows: lanes per candidate group
#ifndef ADD_GRID
#define ADD_GRID 768
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

// Symmetric rows: a 512-thread workgroup owns (row, chunk of kPts = 256 query
// points); its eight one-wave groups scan disjoint eighths of the candidate
// list for the same query points (the first-minimum update is a dependent
// chain, so latency, not issue, bounds a lone wave: 8 waves per item, kPPL = 4
// chains per lane — each broadcast candidate read serves four distances: 155
// -> 148 us against kPPL = 2 on the bench rows — three items per CU), then
// merge in LDS in group order with a strict < —
// a later range wins only with a strictly smaller distance, which is exactly
// the reference's sequential first minimum (cu.cc:150-172).
#ifndef ADD_GROUPS
#define ADD_GROUPS 8
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
                                                           float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float4 gpts[];  // [P] GT-rotated points
  __shared__ float mdist[kSymGroups - 1][kPts];                   // range minima of groups 1..kSymGroups-1
  __shared__ int midx[kSymGroups - 1][kPts];
  __shared__ float red[kSymThreads / 64][5];
  __shared__ int s_imin[kPts];
  const int R = rows_of(num_rois_dev, R_cap);
  const int sym_items = *nsym * nchunk;
  const int items = sym_items + R;  // then one plain item per row (add_plain_row)
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
  int n, chunk;
  if (item < nsym_rows * nfull) {
    n = sym_rows[item / nfull];
    chunk = item % nfull;
  } else {
    n = sym_rows[item - nsym_rows * nfull];
    chunk = nfull;
  }
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
    const float4 cm = gpts[im];
    const float x2 = cm.x, y2 = cm.y, z2 = cm.z;
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

// Row classes once (first class with weight > 0, cu.cc:47-52) and the
// ascending list of symmetric rows (ballot scan, one workgroup: deterministic).
__global__ void __launch_bounds__(1024) k_add_prep(const float* __restrict__ weight, const float* __restrict__ symmetry,
                                                    int R_cap, const int32_t* __restrict__ num_rois_dev, int C,
                                                    int32_t* __restrict__ rcls, int32_t* __restrict__ sym_rows,
                                                    int32_t* __restrict__ nsym, int32_t* __restrict__ queue) {
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

extern "C" size_t pcnn_add_loss_workspace_size(int R_cap, int C, int P) {
  (void)C;
  const int nchunk = (P + kPts - 1) / kPts;
  const size_t R = (size_t)(R_cap > 0 ? R_cap : 1);
  return pcnn::align_up(R * nchunk * 5 * sizeof(float), 256) + 2 * pcnn::align_up(R * sizeof(int32_t), 256) +
         pcnn::align_up(R * sizeof(float), 256) + 3 * 256;
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
  pcnn::Carve cv(workspace);
  float* partial = cv.take<float>((size_t)R_cap * nchunk * 5);
  int32_t* rcls = cv.take<int32_t>(R_cap);
  int32_t* sym_rows = cv.take<int32_t>(R_cap);
  int32_t* nsym = cv.take<int32_t>(1);
  int32_t* queue = cv.take<int32_t>(1);
  float* row_loss = cv.take<float>(R_cap);
  if (!prepared)
    hipLaunchKernelGGL(k_add_prep, dim3(1), dim3(1024), 0, st, weight, symmetry, R_cap, num_rois_dev, C, rcls,
                       sym_rows, nsym, queue);
  // one persistent grid: symmetric (row, chunk) items of the device-side list, then the plain rows
  const long sym_items = (long)R_cap * nchunk + R_cap;  // symmetric (row, chunk) items, then plain rows
  const int sym_grid = (int)(sym_items < ADD_GRID ? sym_items : ADD_GRID);
  hipLaunchKernelGGL(k_add_rows, dim3(sym_grid), dim3(kSymThreads), (size_t)P * sizeof(float4), st, pred,
                     target, weight, points, symmetry, R_cap, num_rois_dev, C, P, margin, loss_norm_rows,
                     loss_norm_rows_dev, nchunk, rcls, sym_rows, nsym, queue, partial);
  hipLaunchKernelGGL(k_add_finish_rows, dim3((R_cap + 3) / 4), dim3(256), 0, st, R_cap, num_rois_dev, C, nchunk,
                     rcls, partial, row_loss, bottom_diff);
  hipLaunchKernelGGL(k_add_total, dim3(1), dim3(1024), 0, st, R_cap, num_rois_dev, row_loss, loss);
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

// The row classification of pcnn_add_loss_fwd on its own: it reads only the
// weights (the Hough op's targets), so a caller can run it as soon as they
// exist, on another stream, off the chain that produces the predictions.
extern "C" int pcnn_add_loss_prep(const float* weight, const float* symmetry, int R_cap, const int32_t* num_rois_dev,
                                  int C, int P, void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(weight && symmetry && workspace && R_cap > 0 && C > 0 && P > 0 && P <= kMaxPointsLds);
  if (workspace_bytes < pcnn_add_loss_workspace_size(R_cap, C, P)) return PCNN_ECAPACITY;
  const int nchunk = (P + kPts - 1) / kPts;
  pcnn::Carve cv(workspace);
  (void)cv.take<float>((size_t)R_cap * nchunk * 5);
  int32_t* rcls = cv.take<int32_t>(R_cap);
  int32_t* sym_rows = cv.take<int32_t>(R_cap);
  int32_t* nsym = cv.take<int32_t>(1);
  int32_t* queue = cv.take<int32_t>(1);
  hipLaunchKernelGGL(k_add_prep, dim3(1), dim3(1024), 0, (hipStream_t)stream, weight, symmetry, R_cap, num_rois_dev,
                     C, rcls, sym_rows, nsym, queue);
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
