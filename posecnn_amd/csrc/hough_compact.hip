// Hough voting, stage 1: per-image, per-class voter lists in canonical order.
//
// The reference compacts label pixels into per-class lists with atomicAdd
// (compute_arrays_kernel, hough_voting_gpu_op.cu.cc:174-187; order is
// scheduling dependent), copies the class sizes to the host to select classes
// with > labelThreshold pixels (:644-678) and then lets every Hough cell read
// every skip-th list entry.  Here one coalesced pass over the label map
// (histogram -> scan -> scatter, wave-aggregated by label with ballots) yields
// the lists in ascending raster order — one legal execution of the reference —
// sampled at list positions 0, skip, 2 skip, ... (cu.cc:269), with the present
// class selection done on the device.  Each sampled voter gathers its
// (u, v, z) once and precomputes d = exp(z), the box threshold T(d)
// (project_box, cu.cc:84-120) and the row-bound slopes of its voting cone.
#include "hough_common.h"

namespace pcnn_hough {

// Per-call accumulators zeroed by the histogram kernels, which precede every
// atomic on them: the argmax keys, the slots' largest box radius and the
// per-(slot, row) sampled-voter counts.
__device__ __forceinline__ void zero_accumulators(int b, int blk, int nblk, int C, int H, HoughWs ws) {
  const int n = C * H;
  int32_t* rc = ws.rowcnt + (size_t)b * n;
  for (int i = blk * (int)blockDim.x + (int)threadIdx.x; i < n; i += nblk * (int)blockDim.x) rc[i] = 0;
  if (blk == 0)
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      ws.key[(size_t)b * C + c] = 0ull;
      ws.kmax[(size_t)b * C + c] = -1;
    }
}

__global__ void __launch_bounds__(kCompactThreads) k_label_hist(const int32_t* __restrict__ label, int HW, int C,
                                                                 int H, HoughWs ws) {
  __shared__ int h[kMaxClasses];
  const int b = blockIdx.y, blk = blockIdx.x;
  for (int i = threadIdx.x; i < C; i += blockDim.x) h[i] = 0;
  zero_accumulators(b, blk, ws.nblk, C, H, ws);
  __syncthreads();
  const int32_t* lab = label + (size_t)b * HW;
  const int base = blk * kPixPerBlk;
  constexpr int kRounds = kPixPerBlk / kCompactThreads;
  int lr[kRounds];  // every round's label load in flight at once
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const int p = base + r * kCompactThreads + threadIdx.x;
    lr[r] = p < HW ? lab[p] : -1;
  }
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const int l = lr[r];
    const bool valid = l > 0 && l < C;
    for_each_label_group(l, valid, [&](int l0, uint64_t m) {
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) atomicAdd(&h[l0], __popcll(m));
    });
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) ws.blk[((size_t)b * ws.nblk + blk) * C + i] = h[i];
}

// k_label_hist with the label producer fused in: the
// block's pixels are labelled by argmax over prob_normalized (argmax_2d,
// network.py:433-434) as they are counted, and label_2d is written once for
// k_label_place (and the caller).  One pass over the (B,H,W,C) prob map
// replaces the argmax pass + label write + label re-read of the unfused graph.
// Dynamic LDS: kCompactThreads/64 waves x 64 px x C floats when C is staged.
__global__ void __launch_bounds__(kCompactThreads) k_label_hist_prob(const float* __restrict__ prob,
                                                                      int32_t* __restrict__ label_out, int HW,
                                                                      int C, int H, HoughWs ws) {
  extern __shared__ __attribute__((aligned(16))) float stage_all[];
  __shared__ int h[kMaxClasses];
  const int b = blockIdx.y, blk = blockIdx.x;
  for (int i = threadIdx.x; i < C; i += blockDim.x) h[i] = 0;
  zero_accumulators(b, blk, ws.nblk, C, H, ws);
  const float* img = prob + (size_t)b * HW * C;
  float* stage = stage_all + (threadIdx.x >> 6) * 64 * (C <= kArgmaxStagedMaxC ? C : 0);
  const int base = blk * kPixPerBlk;
  for (int r = 0; r < kPixPerBlk / kCompactThreads; r++) {
    const int p0 = base + r * kCompactThreads + (threadIdx.x & ~63);
    const int p = p0 + pcnn::lane_id();
    const int l = wave_argmax_rows(img, p0, HW, C, stage);  // syncs the workgroup (h[] init included)
    if (p < HW) label_out[(size_t)b * HW + p] = l;
    const bool valid = p < HW && l > 0;
    for_each_label_group(l, valid, [&](int l0, uint64_t m) {
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) atomicAdd(&h[l0], __popcll(m));
    });
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) ws.blk[((size_t)b * ws.nblk + blk) * C + i] = h[i];
}

// Row-bound setup of one cone (threshold cc, ss = sqrt(1 - cc^2)): the cone is
// {p : cross(m, p) > 0 and cross(p, q) > 0} with m / q the voter direction
// rotated by -/+ acos(cc).  On row dy each constraint is a half-line of dx: a
// slope s with dx > s*dy (lower) or dx < s*dy (upper), or (boundary parallel
// to the row) a sign condition on dy.
__device__ __forceinline__ void bound_setup(double ex, double ey, double cc, double ss, double& s1, int& c1,
                                            double& s2, int& c2) {
  const double qx = ex * cc - ey * ss, qy = ex * ss + ey * cc;  // +theta
  const double mx = ex * cc + ey * ss, my = -ex * ss + ey * cc; // -theta
  // (1) -my * dx > -mx * dy
  s1 = 0.0;
  if (my < 0.0) { c1 = kBoundLower; s1 = mx / my; }
  else if (my > 0.0) { c1 = kBoundUpper; s1 = mx / my; }
  else c1 = mx > 0.0 ? kNeedPosDy : kNeedNegDy;
  // (2) qy * dx > qx * dy
  s2 = 0.0;
  if (qy > 0.0) { c2 = kBoundLower; s2 = qx / qy; }
  else if (qy < 0.0) { c2 = kBoundUpper; s2 = qx / qy; }
  else c2 = qx > 0.0 ? kNeedNegDy : kNeedPosDy;
}

// Cone row-bound slopes and code of one voter (u, v, d, T): the outer / inner
// cone at the inlier threshold -/+ kConeEps (so / si = sqrt(1 - c^2) of each);
// returns the box radius k (-1: votes for no cell).
__device__ __forceinline__ int voter_cone(float4 q, float inlier, double so, double si, float4& cone, int& code) {
  const double c = (double)inlier;
  const bool fast_ok = c > 0.05 && c < 0.999;
  const float u = q.x, v = q.y;
  const float n1f = sqrtf(u * u + v * v);
  double sl[4] = {0.0, 0.0, 0.0, 0.0};
  const int k = box_radius(q.w);
  code = 0;
  if (k < 0) {
    code = kDeadVoter;
  } else if (!fast_ok || !(n1f >= 1e-18f && n1f <= 1e18f)) {
    code = kSlowVoter;
  } else {
    const double ud = u, vd = v;
    const double nd = sqrt(ud * ud + vd * vd);
    const double ex = ud / nd, ey = vd / nd;
    int c0, c1, c2, c3;
    bound_setup(ex, ey, c - kConeEps, so, sl[0], c0, sl[1], c1);  // outer cone
    bound_setup(ex, ey, c + kConeEps, si, sl[2], c2, sl[3], c3);  // inner cone
    code = c0 | (c1 << 2) | (c2 << 4) | (c3 << 6);
  }
  // slopes are evaluated in float per row (hough_vote.hip): the float error
  // of an interval end is <= ~2.6% of the +-kConeEps margin in x there
  auto cl = [](double x) { return (float)(x > 1e30 ? 1e30 : (x < -1e30 ? -1e30 : x)); };
  cone = make_float4(cl(sl[0]), cl(sl[1]), cl(sl[2]), cl(sl[3]));
  return k;
}

// vch = channels per vertex pixel: 3C (the reference's (B,H,W,3C) map, a
// voter reads its class's channels 3l..3l+2) or 3 (the class-compact map of
// the pixel's own class only).
//
// One pass per (pixel block, image) after the histograms: the block's
// exclusive offsets and the class totals from the block histograms (every
// block reads them; no separate scan launch), the present-class selection
// (class c >= 1 with > label_thr pixels, cu.cc:654-664; the first index_size
// vote, cu.cc:775-776) and the voter-list offsets in LDS -- block 0 publishes
// them for the later kernels -- then the ranked scatter of the sampled voters
// (list positions 0, skip, 2 skip, ...: cu.cc:269) with each voter's record
// (u, v, d = exp(z), T(d)), its cone row-bound slopes and code, its (slot,
// row) count and the slot's largest box radius.  The block's sampled voters
// are queued in LDS first and set up in one dense pass (round 5: the setup
// used to run per round on the one lane in ten that samples -- or as a
// kernel of its own, k_voter_setup, 7.8 us at B = 1).
__global__ void __launch_bounds__(kCompactThreads) k_label_place(
    const int32_t* __restrict__ label, const float* __restrict__ vertex, int vch, const float* __restrict__ extents,
    const float* __restrict__ meta, int num_meta, int H, int W, int C, int skip, int label_thr, int index_size,
    int nms, float inlier, double so, double si, HoughWs ws) {
  __shared__ int run[kMaxClasses];
  __shared__ int tot[kMaxClasses];
  __shared__ int vbl[kMaxClasses], vcl[kMaxClasses], slot_of[kMaxClasses], scls[kMaxClasses];
  __shared__ int pe[kCompactThreads], pa[kCompactThreads];
  // dynamic LDS (sized by place_lds_bytes): the (round, wave, class) group
  // counts, then their prefix; the sampled-voter queue (position, class,
  // record slot) of at most place_queue_cap entries
  extern __shared__ int dyn_lds[];
  int* wc = dyn_lds;
  const int qcap = place_queue_cap(C, skip);
  int* qp = wc + (kPixPerBlk / 64) * C;
  int* ql = qp + qcap;
  int* qi = ql + qcap;
  __shared__ int smax[kMaxClasses];  // the block's largest box radius per slot
  __shared__ int s_nq;
  __shared__ int s_nvote, s_count;
  const int b = blockIdx.y, blk = blockIdx.x, nblk = ws.nblk;
  const int HW = H * W;
  const int wave = threadIdx.x >> 6, t = threadIdx.x;
  // 1. exclusive offsets of this block and class totals (G interleaved partial sums per class)
  const int G = kCompactThreads / C > 0 ? kCompactThreads / C : 1;
  if (t < G * C) {
    const int c = t % C, g = t / C;
    int e = 0, a = 0;
    const int* hb = ws.blk + (size_t)b * nblk * C + c;
    int k = g;
    for (; k + 7 * G < nblk; k += 8 * G) {  // eight loads in flight
      int v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) v[u] = hb[(size_t)(k + u * G) * C];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        a += v[u];
        e += k + u * G < blk ? v[u] : 0;
      }
    }
    for (; k < nblk; k += G) {
      const int v = hb[(size_t)k * C];
      a += v;
      e += k < blk ? v : 0;
    }
    pe[t] = e;
    pa[t] = a;
  }
  __syncthreads();
  for (int c = t; c < C; c += blockDim.x) {
    int e = 0, a = 0;
    for (int g = 0; g < G; g++) {
      e += pe[g * C + c];
      a += pa[g * C + c];
    }
    run[c] = e;
    tot[c] = a;
    vbl[c] = 0;
    vcl[c] = 0;
    slot_of[c] = -1;
  }
  __syncthreads();
  // 2. slot table
  if (t == 0) {
    int count = 0;
    for (int c = 1; c < C; c++)
      if (tot[c] > label_thr) scls[count++] = c;
    const int nvote = nms ? count : (count < index_size ? count : index_size);
    int vb = 0;
    for (int sl = 0; sl < nvote; sl++) {
      const int c = scls[sl];
      const int nv = (tot[c] + skip - 1) / skip;
      vbl[c] = vb;
      vcl[c] = nv;
      slot_of[c] = sl;
      vb += nv;
    }
    s_nvote = nvote;
    s_count = count;
    if (blk == 0) {
      if (b == 0)
        for (int i = 0; i < 4; i++) ws.diag[i] = 0;  // self-check counters of this call (pcnn_hough_voting_diag)
      ws.nslots[b] = count;
      ws.nvote[b] = nvote;
      ws.ncand[b] = 0;
      ws.nvtot[b] = vb;
    }
  }
  __syncthreads();
  if (blk == 0)
    for (int c = t; c < C; c += blockDim.x) {
      ws.total[(size_t)b * C + c] = tot[c];
      ws.vbase[(size_t)b * C + c] = vbl[c];
      ws.vcount[(size_t)b * C + c] = vcl[c];
    }
  if (blk == 0)
    for (int sl = t; sl < s_count; sl += blockDim.x) ws.slot_cls[(size_t)b * C + sl] = scls[sl];
  // 3. ranked scatter + voter setup.  The block's labels are loaded up front
  // (kRounds loads in flight per thread), the ranks of every round come from
  // one LDS prefix over (round, wave) group counts, and the sampled voters'
  // vertex gathers are issued together before any of them is used: the
  // rounds no longer wait on each other's global loads.
  constexpr int kRounds = kPixPerBlk / kCompactThreads;
  constexpr int kWaves = kCompactThreads / 64;
  const int32_t* lab = label + (size_t)b * HW;
  const float* mb = meta + (size_t)b * num_meta;
  const int base = blk * kPixPerBlk;
  int lr[kRounds];
#pragma unroll
  for (int rr = 0; rr < kRounds; rr++) {
    const int p = base + rr * kCompactThreads + t;
    lr[rr] = p < HW ? lab[p] : -1;
  }
  for (int i = t; i < kRounds * kWaves * C; i += blockDim.x) wc[i] = 0;
  for (int i = t; i < C; i += blockDim.x) smax[i] = -1;
  if (t == 0) s_nq = 0;
  __syncthreads();
  int rank_w[kRounds];
#pragma unroll
  for (int rr = 0; rr < kRounds; rr++) {
    const int l = lr[rr];
    const bool valid = l > 0 && l < C;
    rank_w[rr] = 0;
    for_each_label_group(l, valid, [&](int l0, uint64_t m) {
      if (l == l0 && valid) rank_w[rr] = __popcll(m & pcnn::lanemask_lt());
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) wc[(rr * kWaves + wave) * C + l0] = __popcll(m);
    });
  }
  __syncthreads();
  // wc -> exclusive prefix over (round, wave) per class, starting at run[c]
  for (int c = t; c < C; c += blockDim.x) {
    int acc = run[c];
    for (int i = 0; i < kRounds * kWaves; i++) {
      const int v = wc[i * C + c];
      wc[i * C + c] = acc;
      acc += v;
    }
  }
  __syncthreads();
  // the sampled voters of the block into an LDS queue (any order: each has
  // its own record slot), then one dense pass of gathers, exp and
  // project_box -- the double exp and the box projection run once per
  // voter, not once per round for every wave holding one
#pragma unroll
  for (int rr = 0; rr < kRounds; rr++) {
    const int l = lr[rr];
    if (l > 0 && l < C && vcl[l] > 0) {
      const int rank = wc[(rr * kWaves + wave) * C + l] + rank_w[rr];
      if (rank % skip == 0) {  // list positions 0, skip, 2 skip, ... (cu.cc:269)
        const int q = atomicAdd(&s_nq, 1);
        qp[q] = base + rr * kCompactThreads + t;
        ql[q] = l;
        qi[q] = vbl[l] + rank / skip;
      }
    }
  }
  __syncthreads();
  const int nq = s_nq;
  int32_t* rowcnt = ws.rowcnt + (size_t)b * C * H;
  for (int q0 = 0; q0 < nq; q0 += blockDim.x) {  // block-uniform trip count
    const int q = q0 + t;
    const bool in = q < nq;
    int k = -1, slot = 0, y = 0;
    if (in) {
      const int p = qp[q], l = ql[q];
      const size_t off = ((size_t)b * HW + p) * (size_t)vch + (vch == 3 ? 0 : 3 * l);
      const float u = vertex[off], v = vertex[off + 1];
      const float d = (float)exp((double)vertex[off + 2]);  // cu.cc:280
      const float T = project_box(l, extents, mb, d, 0.6f);  // cu.cc:285
      const size_t vi = (size_t)b * ws.vcap + qi[q];
      const float4 rec = make_float4(u, v, d, T);
      ws.vdat[vi] = rec;
      ws.vpos[vi] = p;
      // the voter's cone row-bound slopes and code (formerly k_voter_setup)
      float4 cone;
      int code;
      k = voter_cone(rec, inlier, so, si, cone, code);
      ws.vcone[vi] = cone;
      ws.vcode[vi] = code;
      slot = slot_of[l];
      y = p / W;
    }
    // (slot, row) voter counts and the slot's largest box radius, aggregated
    // per wave (queued voters of one row and class sit together)
    for_each_label_group(slot * H + y, in, [&](int key, uint64_t m) {
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) atomicAdd(&rowcnt[key], __popcll(m));
    });
    for_each_label_group(slot, in && k >= 0, [&](int s0, uint64_t m) {
      int kk = (in && k >= 0 && slot == s0) ? k : -1;
      kk = pcnn::wave_max(kk);
      if (pcnn::lane_id() == __ffsll((long long)m) - 1) atomicMax(&smax[s0], kk);
    });
  }
  __syncthreads();
  for (int sl = t; sl < s_nvote; sl += blockDim.x)
    if (smax[sl] >= 0) atomicMax(ws.kmax + (size_t)b * C + sl, smax[sl]);
}

}  // namespace pcnn_hough
