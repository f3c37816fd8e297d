// Hough voting, stage 2: the vote.
//
// Reference: compute_hough_kernel (hough_voting_gpu_op.cu.cc:253-294) — one
// thread per (present class, cell) looping over every sampled voter, with a
// global `hough_space[index]++` per vote: count * H * W * N_c / skip predicate
// evaluations per image.
//
// Here: one workgroup per (band of kBand rows, class slot, image).  For a voter
// and a row r of the band inside its +-T box, the cells (cx, r) satisfying
//   angle_distance(cx, r, x, y, u, v) > 0.9  (cu.cc:32-42, :283)
// form an interval (the cone of half-angle acos(0.9) is convex).  The real
// intervals of an outer and an inner cone (threshold -/+ 2e-6, ~4x the worst
// float error of the reference predicate) bracket it: cells inside the inner
// interval vote, cells outside the outer one do not, and the cells in between
// (usually none) are decided by the reference's float predicate itself.  Each
// run adds +1/-1 to an LDS difference row (integer adds: order-free, exact);
// rows are prefix-summed and the first maximum of the class (thrust
// max_element, cu.cc:757) is folded into one 64-bit atomicMax per workgroup:
// key = count << 32 | ~(y*W + x).
#include "hough_common.h"

namespace pcnn_hough {

// Float is enough here: the outer / inner cones sit +-kConeEps (in cos) from
// the reference threshold, which at row dy is dx = |dy| * 4.6e-6 / sin^2(phi)
// away from the exact boundary (phi = boundary angle to the row); the float
// error of s * dy is |dy * cot(phi)| * 2^-24 (+ the slope's own rounding),
// i.e. at most ~2.6% of that margin.  The bracket stays conservative.
__device__ __forceinline__ bool row_interval(int code1, float s1, int code2, float s2, float dy, float& lo,
                                             float& hi) {
  // branch-free (the codes differ across the lanes of a wave)
  const float b1 = s1 * dy, b2 = s2 * dy;
  lo = fmaxf(code1 == kBoundLower ? b1 : -1e30f, code2 == kBoundLower ? b2 : -1e30f);
  hi = fminf(code1 == kBoundUpper ? b1 : 1e30f, code2 == kBoundUpper ? b2 : 1e30f);
  const bool ok1 = code1 == kNeedPosDy ? dy > 0.f : (code1 == kNeedNegDy ? dy < 0.f : true);
  const bool ok2 = code2 == kNeedPosDy ? dy > 0.f : (code2 == kNeedNegDy ? dy < 0.f : true);
  return ok1 && ok2 && lo < hi;
}

// integer cell range [a, b] of x + dx for dx strictly inside (lo, hi), clipped
__device__ __forceinline__ void int_range(float lo, float hi, int x, int cx0, int cx1, int& a, int& b) {
  lo = fmaxf(lo, -1e9f);
  hi = fminf(hi, 1e9f);
  const int la = (int)floorf(lo) + 1 + x;
  const int lb = (int)ceilf(hi) - 1 + x;
  a = la < cx0 ? cx0 : la;
  b = lb > cx1 ? cx1 : lb;
}

__device__ __forceinline__ void add_run(int* row, int a, int b) {
#ifndef PCNN_ABLATE_ATOMICS
  atomicAdd(&row[a], 1);
  atomicAdd(&row[b + 1], -1);
#else
  if (a == 12345678) row[b] = 1;
#endif
}

// exact reference predicate over cells [a, b] of one row, runs merged
__device__ __forceinline__ void exact_cells(int* row, int a, int b, int r, int x, int y, float u, float v,
                                            float inlier) {
  int start = -1;
  for (int cx = a; cx <= b; cx++) {
    const bool on = cone_pred(cx, r, x, y, u, v, inlier);
    if (on && start < 0) start = cx;
    if (!on && start >= 0) {
      add_run(row, start, cx - 1);
      start = -1;
    }
  }
  if (start >= 0) add_run(row, start, b);
}

// kBand rows x kVoteThreads lanes per workgroup: (4, 512) for B >= 3, (2, 512)
// for B <= 2, where the grid is small and one workgroup's voter loop is the
// critical path.  Measured op times (scripts/vote_ab.sh), B = 1 / 2 / 4 / 8:
// 4 x 512: 88.4 / 121.5 / 131.1 / 169.0 us; 2 x 512: 80.0 / 118.4 / 143.0 /
// 196.1; 2 x 1024: 89.2 / 133.4 / 190.0 / 294.6; 1 x 1024: 112.4 / 178.7 /
// 280.6 / 463.2; 4 x 1024 at B = 1 / 8: 82.2 / 217.0; at B = 4 / 8:
// 4 x 256 150 / 177, 8 x 256 194 / 217, 2 x 256 134 / 173, 3 x 512 133 / 177
// against 131 / 170 for 4 x 512.
template <int kBand, int kVoteThreads>
__global__ void __launch_bounds__(kVoteThreads) k_hough_vote(int H, int W, int C, float inlier, HoughWs ws,
                                                              int32_t* __restrict__ counts_out) {
  extern __shared__ __attribute__((aligned(16))) int diff[];  // [kBand][W + 1]
  __shared__ unsigned long long bkey[kVoteThreads / 64];
  const int b = blockIdx.z, slot = blockIdx.y, band = blockIdx.x;
  if (slot >= ws.nvote[b]) return;
  const int cls = ws.slot_cls[(size_t)b * C + slot];
  const int vb = ws.vbase[(size_t)b * C + cls];
  const int y0 = band * kBand;
  const int y1 = min(y0 + kBand, H);
  const int Wp = W + 1;
  // only voters whose +-k rows can reach the band (rows in [y0 - kmax, y1 - 1 + kmax])
  const int kx = ws.kmax[(size_t)b * C + slot];
  __shared__ int red[2][kVoteThreads / 64];
  int ibeg = 0, iend = 0;
  if (kx >= 0) {  // block-uniform: voters in rows < ylo and < yhi1 of the raster-ordered list
    const int32_t* rc = ws.rowcnt + ((size_t)b * C + slot) * H;
    const int ylo = max(0, y0 - kx), yhi1 = (int)min((long)H, (long)y1 + kx);  // rows [ylo, yhi1)
    int a = 0, c = 0;
    for (int r = threadIdx.x; r < yhi1; r += blockDim.x) {
      const int v = rc[r];
      a += r < ylo ? v : 0;
      c += v;
    }
    a = pcnn::wave_sum(a);
    c = pcnn::wave_sum(c);
    if (pcnn::lane_id() == 0) {
      red[0][threadIdx.x >> 6] = a;
      red[1][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    for (int w = 0; w < kVoteThreads / 64; w++) {
      ibeg += red[0][w];
      iend += red[1][w];
    }
  }
  if (ibeg >= iend && !counts_out) {
    // no voter reaches the band: all its counts are 0; its first-max key is
    // (0, first cell) — needed only when the whole slot has no vote
    if (threadIdx.x == 0) atomicMax(ws.key + (size_t)b * C + slot, 0xFFFFFFFFull - (unsigned)(y0 * W));
    return;
  }
  for (int i = threadIdx.x; i < kBand * Wp; i += blockDim.x) diff[i] = 0;
  __syncthreads();

  const size_t v0 = (size_t)b * ws.vcap + vb;
  // the next voter's record is loaded while the current one is processed
  int i = ibeg + (int)threadIdx.x;
  float4 qn = make_float4(0.f, 0.f, 0.f, 0.f), sn = qn;
  int pn = 0, cn = 0;
  if (i < iend) {
    qn = ws.vdat[v0 + i];
    pn = ws.vpos[v0 + i];
    cn = ws.vcode[v0 + i];
    sn = ws.vcone[v0 + i];
  }
  for (; i < iend; i += blockDim.x) {
    const float4 q = qn, s = sn;
    const int p = pn, code = cn;
    if (i + (int)blockDim.x < iend) {
      const size_t jn = v0 + i + blockDim.x;
      qn = ws.vdat[jn];
      pn = ws.vpos[jn];
      cn = ws.vcode[jn];
      sn = ws.vcone[jn];
    }
    const int x = p % W, y = p / W;
    const int k = box_radius(q.w);
    if (k < 0) continue;
    const int ry0 = max(y - k, y0), ry1 = min(y + k, y1 - 1);
    if (ry0 > ry1) continue;
#ifdef PCNN_ABLATE_ROWS
    if (ry0 == -12345) diff[0] = 1;
    continue;
#endif
    const int bx0 = max(x - k, 0), bx1 = min(x + k, W - 1);
    const float u = q.x, v = q.y;
    if (code & kSlowVoter) {  // pathological direction / threshold: exact predicate everywhere
      for (int r = ry0; r <= ry1; r++) exact_cells(diff + (r - y0) * Wp, bx0, bx1, r, x, y, u, v, inlier);
      continue;
    }
    const int co1 = code & 3, co2 = (code >> 2) & 3, ci1 = (code >> 4) & 3, ci2 = (code >> 6) & 3;
    for (int r = ry0; r <= ry1; r++) {
      int* row = diff + (r - y0) * Wp;
      const float dy = (float)(r - y);
      float lo, hi;
      if (!row_interval(co1, s.x, co2, s.y, dy, lo, hi)) continue;
      int oa, ob;
      int_range(lo, hi, x, bx0, bx1, oa, ob);
      if (oa > ob) continue;
      int ia = 1, ib = 0;
#ifdef PCNN_ABLATE_INNER
      ia = oa; ib = ob;
      if (false) {
#else
      if (row_interval(ci1, s.z, ci2, s.w, dy, lo, hi)) {
#endif
        int_range(lo, hi, x, bx0, bx1, ia, ib);
        ia = max(ia, oa);
        ib = min(ib, ob);
      }
      if (ia <= ib) {
        add_run(row, ia, ib);
#ifndef PCNN_ABLATE_EXACT
        if (oa < ia) exact_cells(row, oa, ia - 1, r, x, y, u, v, inlier);
        if (ib < ob) exact_cells(row, ib + 1, ob, r, x, y, u, v, inlier);
      } else {
        exact_cells(row, oa, ob, r, x, y, u, v, inlier);
#endif
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

template __global__ void k_hough_vote<4, 512>(int, int, int, float, HoughWs, int32_t*);
template __global__ void k_hough_vote<2, 512>(int, int, int, float, HoughWs, int32_t*);

}  // namespace pcnn_hough
