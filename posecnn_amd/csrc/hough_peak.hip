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
  __shared__ int wcnt[kPeakThreads / 64];
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // Voters that vote for (cx, cy) are compacted in voter order into sh_d
  // (ballot ranks + per-wave offsets); the others would add +0.0f to a
  // non-negative sum, which leaves it unchanged, so thread 0's in-order sum
  // over the compacted terms equals the reference's loop (cu.cc:269-294).
  int start = 0;
  while (start < nv) {
    int fill = 0;  // compacted terms in sh_d (block-uniform)
    int j0 = start;
    for (; j0 < nv && fill + (int)blockDim.x <= kPeakChunk; j0 += blockDim.x) {
      const int j = j0 + threadIdx.x;
      bool f = false;
      float d = 0.f;
      if (j < nv) {
        const float4 q = vd[j];
        const int p = vp[j];
        const int x = p % W, y = p / W;
        f = cone_pred(cx, cy, x, y, q.x, q.y, inlier);
        if (f) {
          float dx = fabsf((float)(x - cx));
          float dy = fabsf((float)(y - cy));
          f = dx < q.w && dy < q.w;  // cu.cc:288
        }
        d = q.z;
      }
      const uint64_t m = __ballot(f);
      if (lane == 0) wcnt[wave] = __popcll(m);
      __syncthreads();
      int off = fill;
      for (int w = 0; w < wave; w++) off += wcnt[w];
      if (f) sh_d[off + __popcll(m & pcnn::lanemask_lt())] = d;
      int tot = 0;
      for (int w = 0; w < nw; w++) tot += wcnt[w];
      cnt += f ? 1 : 0;
      fill += tot;
      __syncthreads();
    }
    start = j0;
    if (threadIdx.x == 0) {  // distance += d in voter order (cu.cc:291), reads prefetched ahead of the adds
      int i = 0;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      if (fill >= 4) { a0 = sh_d[0]; a1 = sh_d[1]; a2 = sh_d[2]; a3 = sh_d[3]; }
      for (; i + 8 <= fill; i += 4) {
        const float b0 = sh_d[i + 4], b1 = sh_d[i + 5], b2 = sh_d[i + 6], b3 = sh_d[i + 7];
        dsum += a0; dsum += a1; dsum += a2; dsum += a3;
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
      }
      if (i + 4 <= fill) {
        dsum += a0; dsum += a1; dsum += a2; dsum += a3;
        i += 4;
      }
      for (; i < fill; i++) dsum += sh_d[i];
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

// ---------------------------------------------------------------------------
// The same cell, with the reference's in-order fp32 sum (cu.cc:269-291)
// computed in parallel and bit for bit (round 5).  The serial chain
// s_k = fl(s_{k-1} + d_k) over the voting voters is one dependent add per
// term; here every thread holds a contiguous run of the voters in registers
// and the chain is rebuilt from three facts about fp32 addition of a
// non-negative term to a non-negative running sum:
//  - while s stays in one binade [2^E, 2^(E+1)), s is an integer S times
//    u = 2^(E-23) and fl(s + d) = (S + r) u, where r = round(d / u) to nearest
//    and, on an exact half, r is chosen so that S + r is even: r depends on S
//    only through its parity.  A term is a two-entry "transducer" (the
//    increment for S even / odd), and transducers compose associatively, so
//    a run of terms in one binade is one block scan;
//  - the binade of every partial sum is predicted from the exact prefix sums
//    (double); each term where the predicted binade changes (a crossing, and
//    the first term) is an event, added by one lane with the real fp32 add
//    from the exact running sum, so its rounding is the reference's;
//  - every prediction is then verified: each in-binade term must keep
//    S in [2^23, 2^24) and each event must land in the binade predicted for
//    the run that follows it.  If all hold, the partial sums are the serial
//    ones by induction; if one fails (a prefix within rounding of a power of
//    two, a non-finite term, more than kPsumEvents events or more than
//    kPsumPer voters per thread), the caller falls back to exact_cell's
//    serial chain.  The bb pass then uses the cached cone flags and |dx|,
//    |dy| (no second read of the voters).
// diag[3] counts the maxima that took that fallback.
// The per-thread voter arrays are unrolled register arrays; the kernel picks
// the smallest instantiation that holds the cell (kPsumPer voters per thread
// is the largest), because the code executed once per cell is what costs:
// at 24 per thread the kernel was 62 KB of straight-line code, and a
// workgroup that runs through it once mostly waits on instruction fetch.
constexpr int kPsumPer = 24;      // voters per thread held in registers (nv <= kPsumPer * kPeakThreads)
constexpr int kPsumSmall = 8;     // the small instantiation
constexpr int kPsumEvents = 256;  // crossing events per cell
constexpr int kPsumBatch = 8;     // phase A voters loaded per batch

struct PsumTr {  // running-sum transducer: increment for S even / odd; has = the run starts at an event
  int i0, i1, has;
};
__device__ __forceinline__ PsumTr psum_id() { return PsumTr{0, 0, 0}; }
// a then b
__device__ __forceinline__ PsumTr psum_cat(const PsumTr& a, const PsumTr& b) {
  if (b.has) return b;
  PsumTr c;
  c.i0 = a.i0 + (((a.i0) & 1) ? b.i1 : b.i0);
  c.i1 = a.i1 + (((1 + a.i1) & 1) ? b.i1 : b.i0);
  c.has = a.has;
  return c;
}
// the transducer of adding q = d / u (exact) to an integer S (no binade change)
__device__ __forceinline__ PsumTr psum_term(float q) {
  const float fl = floorf(q), fr = q - fl;
  const int f = (int)fl;
  PsumTr t;
  t.has = 0;
  if (fr > 0.5f) {
    t.i0 = t.i1 = f + 1;
  } else if (fr < 0.5f) {
    t.i0 = t.i1 = f;
  } else {  // exact half: the even sum
    t.i0 = f + (f & 1);
    t.i1 = f + ((f + 1) & 1);
  }
  return t;
}
// ilogb of a positive finite double (v_frexp_exp); 0 -> a sentinel that is
// neither an exponent nor the -100000 of 'no partial sum yet'
__device__ __forceinline__ int dlogb(double x) { return x > 0.0 ? __builtin_amdgcn_frexp_exp(x) - 1 : -200000; }
__device__ __forceinline__ int f32_binade(float s) {  // E of a positive normal float, -1000 otherwise
  const unsigned b = __float_as_uint(s);
  const int e = (int)((b >> 23) & 0xFF);
  return (e == 0 || e == 255 || (b >> 31)) ? -1000 : e - 127;
}

struct PsumShared {
  float ev_d[kPsumEvents];
  int ev_E[kPsumEvents], ev_i0[kPsumEvents], ev_i1[kPsumEvents], ev_S[kPsumEvents];
  PsumTr wtr[kPeakThreads / 64];
  int wcnt[kPeakThreads / 64], wev[kPeakThreads / 64];
  double wsum[kPeakThreads / 64];
  int fail, total_cnt, total_ev, bbw, bbh;
  float dist;
  PsumTr final_tr;
};

// Returns true with o filled, or false (block-uniform) when the caller must
// take exact_cell's serial path.
template <int kPer>
__device__ bool exact_cell_par(int cx, int cy, int cls, float count_f, const float4* __restrict__ vd,
                               const int32_t* __restrict__ vp, int nv, int W, float inlier,
                               PsumShared& sh, float pre, float gpre, int ngpre, float* s_pre, float* s_gt,
                               PeakOut& o) {
  const int nt = blockDim.x, t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6, nw = nt >> 6;
  constexpr int kBatch = kPer < kPsumBatch ? kPer : kPsumBatch;
  const float rcpW = 1.f / (float)W;
  const int m = (nv + nt - 1) / nt;
  if (m > kPer) return false;  // block-uniform
  const int j0 = t * m;
  // phase A: the thread's voters -> voting flags, d, and the cone voters' |dx|, |dy|;
  // a batch's loads are all issued before its first use (one memory latency
  // per kBatch voters, not one per voter)
  float dd[kPer];
  unsigned pk[kPer];
  unsigned vbits = 0;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    dd[i] = 0.f;
    pk[i] = 0xFFFFFFFFu;
  }
#pragma unroll
  for (int i0 = 0; i0 < kPer; i0 += kBatch) {
    if (i0 >= m) break;  // block-uniform
    float4 q[kBatch];
    int p[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; k++) {
      const int j = j0 + i0 + k;
      const bool live = i0 + k < m && j < nv;
      q[k] = live ? vd[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      p[k] = live ? vp[j] : -1;
    }
#pragma unroll
    for (int k = 0; k < kBatch; k++) {
      const int i = i0 + k;
      if (p[k] >= 0) {
        int y = __float2int_rz((float)p[k] * rcpW), x = p[k] - y * W;  // y = p / W up to a small error, fixed up
        while (x < 0) { y--; x += W; }
        while (x >= W) { y++; x -= W; }
        if (cone_pred(cx, cy, x, y, q[k].x, q[k].y, inlier)) {
          const int adx = abs(x - cx), ady = abs(y - cy);
          pk[i] = (unsigned)adx | ((unsigned)ady << 16);
          if ((float)adx < q[k].w && (float)ady < q[k].w) {  // cu.cc:285-288
            vbits |= 1u << i;
            dd[i] = q[k].z;
            bad |= !(q[k].z >= 0.f) || !isfinite(q[k].z);
          }
        }
      }
    }
  }
  // the bb pass's class extents / camera row and the emit's GT rows, loaded
  // by the caller before the voters (their latency is behind phase A's)
  if (t < 9) s_pre[t] = pre;
  if (t < ngpre) s_gt[t] = gpre;
  // scan 1: voting counts and exact-ish prefix sums (double) -> binade predictions
  int c = __popc(vbits);
  double D = 0.0;
#pragma unroll
  for (int i = 0; i < kPer; i++) D += (double)dd[i];
  int ci = c;
  double Di = D;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const int cy_ = __shfl_up(ci, k, 64);
    const double dy_ = __shfl_up(Di, k, 64);
    if (lane >= k) { ci += cy_; Di += dy_; }
  }
  if (lane == 63) { sh.wcnt[wave] = ci; sh.wsum[wave] = Di; }
  if (t == 0) sh.fail = 0;
  __syncthreads();
  int cbase = ci - c;
  double Pbase = Di - D;
#pragma unroll
  for (int w = 0; w < kPeakThreads / 64; w++) {  // independent LDS reads, summed in wave order
    const int cw = sh.wcnt[w];
    const double sw = sh.wsum[w];
    if (w < wave) { cbase += cw; Pbase += sw; }
  }
  if (t == nt - 1) sh.total_cnt = cbase + c;
  // phase B: events and the thread's tail transducer (terms after its last event)
  PsumTr tail = psum_id();
  int nev = 0;
  {
    double P = Pbase;
    int Eprev = cbase > 0 ? dlogb(Pbase) : -100000;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      if (vbits & (1u << i)) {
        P += (double)dd[i];
        const int E = P > 0.0 ? dlogb(P) : -100000;
        if (E != Eprev) {  // first term or a predicted crossing: an event
          nev++;
          tail = PsumTr{0, 0, 1};
        } else {
          const float q = ldexpf(dd[i], 23 - E);
          bad |= !(q < 8388608.f);
          tail = psum_cat(tail, psum_term(q));
        }
        Eprev = E;
      }
    }
  }
  // scan 2: event counts and the segmented transducer composition
  PsumTr ti = tail;
  int ei = nev;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    PsumTr y;
    y.i0 = __shfl_up(ti.i0, k, 64);
    y.i1 = __shfl_up(ti.i1, k, 64);
    y.has = __shfl_up(ti.has, k, 64);
    const int ey = __shfl_up(ei, k, 64);
    if (lane >= k) { ti = psum_cat(y, ti); ei += ey; }
  }
  if (lane == 63) { sh.wtr[wave] = ti; sh.wev[wave] = ei; }
  if (bad) sh.fail = 1;
  __syncthreads();
  PsumTr X = psum_id();
  int ebase = 0;
#pragma unroll
  for (int w = 0; w < kPeakThreads / 64; w++) {
    const PsumTr tw = sh.wtr[w];
    const int ew = sh.wev[w];
    if (w < wave) { X = psum_cat(X, tw); ebase += ew; }
  }
  {  // exclusive within the wave
    PsumTr y;
    y.i0 = __shfl_up(ti.i0, 1, 64);
    y.i1 = __shfl_up(ti.i1, 1, 64);
    y.has = __shfl_up(ti.has, 1, 64);
    const int ey = __shfl_up(ei, 1, 64);
    if (lane >= 1) { X = psum_cat(X, y); ebase += ey; }
  }
  if (t == nt - 1) {
    sh.final_tr = psum_cat(X, tail);
    sh.total_ev = ebase + nev;
  }
  // phase C: event records (d, predicted binade, the transducer of the run before it)
  {
    PsumTr tr = X;
    double P = Pbase;
    int Eprev = cbase > 0 ? dlogb(Pbase) : -100000;
    int e = ebase;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      if (vbits & (1u << i)) {
        P += (double)dd[i];
        const int E = P > 0.0 ? dlogb(P) : -100000;
        if (E != Eprev) {
          if (e < kPsumEvents) {
            sh.ev_d[e] = dd[i];
            sh.ev_E[e] = E;
            sh.ev_i0[e] = tr.i0;
            sh.ev_i1[e] = tr.i1;
          }
          e++;
          tr = psum_id();
        } else {
          tr = psum_cat(tr, psum_term(ldexpf(dd[i], 23 - E)));
        }
        Eprev = E;
      }
    }
  }
  __syncthreads();
  const int total = sh.total_cnt;
  o.mismatch = ((float)total != count_f) ? 1 : 0;
  o.count = count_f;
  o.distance = 0.f;
  o.bbh2 = 0.f;
  o.bbw2 = 0.f;
  if (!(count_f > 0.f)) return true;  // hough_data stays memset-zero (cu.cc:296, :698-708)
  if (total == 0 || sh.fail || sh.total_ev > kPsumEvents) return false;
  // the walk: the events' fp32 adds in order from the exact running sum.  Wave
  // 0 holds 64 events per pass in its lanes and runs the chain wave-uniformly
  // (operands by readlane, the carried S / E in registers); lane k keeps the
  // k-th event's S for phase D.
  if (wave == 0) {
    float s = 0.f;
    int fail = 0, Sp = 0, Ep = 0;
    const int ne = sh.total_ev;
    for (int e0 = 0; e0 < ne; e0 += 64) {
      const int el = e0 + lane;
      const bool lv = el < ne;
      const float ld = lv ? sh.ev_d[el] : 0.f;
      const int lE = lv ? sh.ev_E[el] : 0, l0 = lv ? sh.ev_i0[el] : 0, l1 = lv ? sh.ev_i1[el] : 0;
      int myS = 0;
      const int n = min(64, ne - e0);
      for (int k = 0; k < n; k++) {
        if (e0 + k > 0) {
          const int inc0 = __builtin_amdgcn_readlane(l0, k), inc1 = __builtin_amdgcn_readlane(l1, k);
          int S = Sp + ((Sp & 1) ? inc1 : inc0);
          fail |= !(S >= (1 << 23) && S < (1 << 24));
          s = ldexpf((float)S, Ep - 23);
        }
        s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ld), k));  // cu.cc:291, in order
        const int E = __builtin_amdgcn_readlane(lE, k);
        fail |= f32_binade(s) != E;
        Sp = (int)ldexpf(s, 23 - E);
        Ep = E;
        if (lane == k) myS = Sp;
      }
      if (lv) sh.ev_S[el] = myS;
    }
    if (ne > 0) {
      const PsumTr ft = sh.final_tr;
      const int S = Sp + ((Sp & 1) ? ft.i1 : ft.i0);
      fail |= !(S >= (1 << 23) && S < (1 << 24));
      s = ldexpf((float)S, Ep - 23);
    }
    fail |= ne == 0;
    if (lane == 0) {
      sh.fail = fail;
      sh.dist = s / count_f;  // cu.cc:298
      sh.bbw = -1;
      sh.bbh = -1;
    }
  }
  __syncthreads();
  if (sh.fail) return false;
  // phase D: verify every in-binade term of the thread (S stays in [2^23, 2^24))
  {
    bool ok = true;
    if (c > 0) {
      int S = 0, E = 0;
      double P = Pbase;
      int Eprev = cbase > 0 ? dlogb(Pbase) : -100000;
      if (cbase > 0 && ebase > 0) {  // the run continues from the last event before this thread
        S = sh.ev_S[ebase - 1];
        E = sh.ev_E[ebase - 1];
        S += (S & 1) ? X.i1 : X.i0;  // X: the terms between that event and this thread
        ok &= S >= (1 << 23) && S < (1 << 24);
      } else if (cbase > 0) {
        ok = false;
      }
      int e = ebase;
#pragma unroll
      for (int i = 0; i < kPer; i++) {
        if (vbits & (1u << i)) {
          P += (double)dd[i];
          const int Ep = P > 0.0 ? dlogb(P) : -100000;
          if (Ep != Eprev) {
            S = sh.ev_S[e];
            E = sh.ev_E[e];
            e++;
          } else {
            const PsumTr tr = psum_term(ldexpf(dd[i], 23 - E));
            S += (S & 1) ? tr.i1 : tr.i0;
            ok &= S >= (1 << 23) && S < (1 << 24);
          }
          Eprev = Ep;
        }
      }
    }
    if (!ok) sh.fail = 1;
  }
  // bb extent with T(distance) over the cached cone voters (cu.cc:300-330),
  // in the same phase as the check (discarded if the check failed)
  const float distance = sh.dist;
  const float Tm = project_box(0, s_pre, s_pre + 3, distance, 0.6f);  // cu.cc:317 (s_pre: the class's row)
  int bw = -1, bh = -1;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    if (pk[i] != 0xFFFFFFFFu) {
      const int adx = (int)(pk[i] & 0xFFFFu), ady = (int)(pk[i] >> 16);
      if ((float)adx < Tm && (float)ady < Tm) {
        bw = max(bw, adx);
        bh = max(bh, ady);
      }
    }
  }
  bw = pcnn::wave_max(bw);
  bh = pcnn::wave_max(bh);
  if (lane == 0 && bw >= 0) atomicMax(&sh.bbw, bw);
  if (lane == 0 && bh >= 0) atomicMax(&sh.bbh, bh);
  __syncthreads();
  if (sh.fail) return false;
  o.distance = distance;
  o.bbw2 = 2 * (float)sh.bbw;
  o.bbh2 = 2 * (float)sh.bbh;
  __syncthreads();  // sh is reused by the caller's next cell
  (void)nw;
  return true;
}

// Default path: one workgroup per (slot, image) = one maximum.  Exact
// hough_data at the argmax, then the slot's RoI rows (emit_max) at output row
// (rows of images < b) + slot * rpm: image-major, ascending slot order.
// Workgroup (0, 0) also writes the row count (+ dummy row) for the batch.
__global__ void __launch_bounds__(kPeakThreads) k_hough_peak(int B, int H, int W, int C, float inlier,
                                                              const float* __restrict__ extents,
                                                              const float* __restrict__ meta, int num_meta,
                                                              HoughWs ws, int is_train, int batch_base,
                                                              const float* __restrict__ gt, int num_gt,
                                                              float* __restrict__ top_box,
                                                              float* __restrict__ top_pose,
                                                              float* __restrict__ top_target,
                                                              float* __restrict__ top_weight,
                                                              int32_t* __restrict__ top_domain,
                                                              int32_t* __restrict__ num_rois, int cap, int psum) {
  __shared__ __attribute__((aligned(16))) float sh_d[kPeakChunk + 4];
  __shared__ float sh_red[2 * (kPeakThreads / 64)];
  __shared__ int s_off[2];
  __shared__ EmitShared esh;
  __shared__ PsumShared psh;
  __shared__ float s_pre[9];             // extents[cls][0..2], meta[0..5] of the image
  __shared__ float s_gt[kPeakThreads];  // the GT rows (train mode, num_gt * 13 <= kPeakThreads)
  const int b = blockIdx.y, slot = blockIdx.x;
  const int rpm = is_train ? 9 : 1;
  if (slot == 0 && b == 0) {  // batch row count: sum over images of nvote * rpm
    if (threadIdx.x == 0) s_off[1] = 0;
    __syncthreads();
    int t = 0;
    for (int i = threadIdx.x; i < B; i += blockDim.x) t += ws.nvote[i] * rpm;
    if (t) atomicAdd(&s_off[1], t);
    __syncthreads();
    emit_count(s_off[1], cap, C, top_box, top_pose, top_target, top_weight, top_domain, num_rois);
  }
  if (slot >= ws.nvote[b]) return;
  if (threadIdx.x == 0) s_off[0] = 0;
  __syncthreads();
  {
    int t = 0;
    for (int i = threadIdx.x; i < b; i += blockDim.x) t += ws.nvote[i] * rpm;
    if (t) atomicAdd(&s_off[0], t);
  }
  const int cls = ws.slot_cls[(size_t)b * C + slot];
  const unsigned long long key = ws.key[(size_t)b * C + slot];
  const unsigned cnt = (unsigned)(key >> 32);
  const unsigned idx = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
  const int cx = (int)(idx % (unsigned)W), cy = (int)(idx / (unsigned)W);
  const int vb = ws.vbase[(size_t)b * C + cls];
  const int nv = ws.vcount[(size_t)b * C + cls];
  const float* mb = meta + (size_t)b * num_meta;
  const float4* vd = ws.vdat + (size_t)b * ws.vcap + vb;
  const int32_t* vpp = ws.vpos + (size_t)b * ws.vcap + vb;
  // what the bb pass and the emit read, loaded now and parked in LDS once the
  // voters have arrived (exact_cell_par, or below on the serial path)
  const int t = threadIdx.x;
  const float pre = t < 3 ? extents[cls * 3 + t] : (t < 9 ? mb[t - 3] : 0.f);
  const int ngpre = is_train && num_gt * 13 <= kPeakThreads ? num_gt * 13 : 0;
  const float gpre = t < ngpre ? gt[t] : 0.f;
  PeakOut o;
  const int mper = (nv + kPeakThreads - 1) / kPeakThreads;
  if (!(psum && (mper <= kPsumSmall
                     ? exact_cell_par<kPsumSmall>(cx, cy, cls, (float)cnt, vd, vpp, nv, W, inlier, psh, pre, gpre,
                                                  ngpre, s_pre, s_gt, o)
                     : exact_cell_par<kPsumPer>(cx, cy, cls, (float)cnt, vd, vpp, nv, W, inlier, psh, pre, gpre,
                                                ngpre, s_pre, s_gt, o)))) {
    o = exact_cell(cx, cy, cls, (float)cnt, vd, vpp, nv, W, inlier, extents, mb, sh_d, sh_red);
    if (psum && threadIdx.x == 0) atomicAdd(&ws.diag[3], 1);  // took the serial chain
  }
  if (t < 9) s_pre[t] = pre;
  if (t < ngpre) s_gt[t] = gpre;
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
  __syncthreads();  // s_off[0] complete
  // two call sites, so that each inlined copy sees one address space for the
  // GT rows: LDS reads (ds_read) do not wait for this wave's earlier global
  // stores the way generic (flat) reads of a mixed pointer would
  if (ngpre)
    emit_max(esh, s_off[0] + slot * rpm, cap, batch_base + b, cls, o.count, o.distance, o.bbh2, o.bbw2, cx, cy,
             is_train, C, s_pre, s_pre + 3, s_gt, num_gt, top_box, top_pose, top_target, top_weight, top_domain,
             ws.diag);
  else
    emit_max(esh, s_off[0] + slot * rpm, cap, batch_base + b, cls, o.count, o.distance, o.bbh2, o.bbw2, cx, cy,
             is_train, C, s_pre, s_pre + 3, gt, num_gt, top_box, top_pose, top_target, top_weight, top_domain,
             ws.diag);
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
                                                                   HoughWs ws, int psum) {
  __shared__ __attribute__((aligned(16))) float sh_d[kPeakChunk + 4];
  __shared__ float sh_red[2 * (kPeakThreads / 64)];
  __shared__ PsumShared psh;
  __shared__ float s_pre[9];
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
    const float4* vd = ws.vdat + (size_t)b * ws.vcap + vb;
    const int32_t* vpp = ws.vpos + (size_t)b * ws.vcap + vb;
    const float* mb = meta + (size_t)b * num_meta;
    const int t = threadIdx.x;
    const float pre = t < 3 ? extents[cls * 3 + t] : (t < 9 ? mb[t - 3] : 0.f);
    PeakOut o;
    const int mper = (nv + kPeakThreads - 1) / kPeakThreads;
    if (!(psum && (mper <= kPsumSmall
                       ? exact_cell_par<kPsumSmall>(cell % W, cell / W, cls, cnt, vd, vpp, nv, W, inlier, psh, pre,
                                                    0.f, 0, s_pre, nullptr, o)
                       : exact_cell_par<kPsumPer>(cell % W, cell / W, cls, cnt, vd, vpp, nv, W, inlier, psh, pre,
                                                  0.f, 0, s_pre, nullptr, o)))) {
      o = exact_cell(cell % W, cell / W, cls, cnt, vd, vpp, nv, W, inlier, extents, mb, sh_d, sh_red);
      if (psum && threadIdx.x == 0) atomicAdd(&ws.diag[3], 1);
    }
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
