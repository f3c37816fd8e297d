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

// k_label_hist with the label producer fused in: the
// block's pixels are labelled by argmax over prob_normalized (argmax_2d,
// network.py:433-434) as they are counted, and label_2d is written once for
// k_label_scatter (and the caller).  One pass over the (B,H,W,C) prob map
// replaces the argmax pass + label write + label re-read of the unfused graph.
// Dynamic LDS: kCompactThreads/64 waves x 64 px x C floats when C is staged.
__global__ void __launch_bounds__(kCompactThreads) k_label_hist_prob(const float* __restrict__ prob,
                                                                      int32_t* __restrict__ label_out, int HW,
                                                                      int C, HoughWs ws) {
  extern __shared__ __attribute__((aligned(16))) float stage_all[];
  __shared__ int h[kMaxClasses];
  const int b = blockIdx.y, blk = blockIdx.x;
  for (int i = threadIdx.x; i < C; i += blockDim.x) h[i] = 0;
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

constexpr int kScanLds = 16384;

// Exclusive scan of the block histograms per class, present-class selection
// (class c >= 1 with > label_thr pixels, cu.cc:654-664) and voter offsets.
__global__ void __launch_bounds__(1024) k_label_scan(int C, int label_thr, int index_size, int nms, int skip,
                                                      HoughWs ws) {
  __shared__ int tile[kScanLds];
  __shared__ int tot[kMaxClasses];
  const int b = blockIdx.x;
  const int n = ws.nblk * C;
  int32_t* hb = ws.blk + (size_t)b * n;
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (n <= kScanLds) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) tile[i] = hb[i];
    __syncthreads();
    for (int c = wave; c < C; c += nw) {
      int run = 0;
      for (int k0 = 0; k0 < ws.nblk; k0 += 64) {
        const int k = k0 + lane;
        const int v = k < ws.nblk ? tile[k * C + c] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          int t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        if (k < ws.nblk) tile[k * C + c] = run + incl - v;
        run += __shfl(incl, 63, 64);
      }
      if (lane == 0) tot[c] = run;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) hb[i] = tile[i];
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      int run = 0;
      for (int k = 0; k < ws.nblk; k++) {
        int v = hb[(size_t)k * C + c];
        hb[(size_t)k * C + c] = run;
        run += v;
      }
      tot[c] = run;
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    ws.total[(size_t)b * C + c] = tot[c];
    ws.key[(size_t)b * C + c] = 0ull;
    ws.kmax[(size_t)b * C + c] = -1;
    ws.vcount[(size_t)b * C + c] = 0;
    ws.vbase[(size_t)b * C + c] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (b == 0)
      for (int i = 0; i < 4; i++) ws.diag[i] = 0;  // self-check counters of this call (pcnn_hough_voting_diag)
    int count = 0;
    for (int c = 1; c < C; c++)
      if (tot[c] > label_thr) ws.slot_cls[(size_t)b * C + count++] = c;
    int nvote = nms ? count : (count < index_size ? count : index_size);  // cu.cc:775-776
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
    ws.nvtot[b] = vb;
  }
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

// vch = channels per vertex pixel: 3C (the reference's (B,H,W,3C) map, a
// voter reads its class's channels 3l..3l+2) or 3 (the class-compact map of
// the pixel's own class only).
__global__ void __launch_bounds__(kCompactThreads) k_label_scatter(const int32_t* __restrict__ label,
                                                                    const float* __restrict__ vertex, int vch,
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
        const size_t vi = (size_t)b * ws.vcap + ws.vbase[(size_t)b * C + l] + rank / skip;
        const size_t off = ((size_t)b * HW + p) * (size_t)vch + (vch == 3 ? 0 : 3 * l);
        const float u = vertex[off], v = vertex[off + 1];
        const float d = (float)exp((double)vertex[off + 2]);  // cu.cc:280
        const float T = project_box(l, extents, mb, d, 0.6f);  // cu.cc:285
        ws.vdat[vi] = make_float4(u, v, d, T);
        ws.vpos[vi] = p;
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

// Cone row-bound slopes of every voter (one thread per voter): outer / inner
// cone at the inlier threshold -/+ kConeEps (so / si = sqrt(1 - c^2) of each).
// Also the per-slot row index of the (raster-ordered) voter list, rowstart[r]
// = first voter with row >= r for rows r in [yfirst, ylast] (yspan), and the
// slot's largest box radius: a vote band [y0, y1) then only visits voters
// with rows in [y0 - kmax, y1 - 1 + kmax].
__global__ void __launch_bounds__(256) k_voter_setup(int H, int W, int C, float inlier, double so, double si,
                                                      HoughWs ws) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < ws.nvtot[b];
  int k = -1, kslot = 0;
  if (in) {
    const size_t vi = (size_t)b * ws.vcap + i;
    const float4 q = ws.vdat[vi];
    const double c = (double)inlier;
    const bool fast_ok = c > 0.05 && c < 0.999;
    const float u = q.x, v = q.y;
    const float n1f = sqrtf(u * u + v * v);
    int code = 0;
    double sl[4] = {0.0, 0.0, 0.0, 0.0};
    k = box_radius(q.w);
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
    auto cl = [](double v) { return (float)(v > 1e30 ? 1e30 : (v < -1e30 ? -1e30 : v)); };
    ws.vcone[vi] = make_float4(cl(sl[0]), cl(sl[1]), cl(sl[2]), cl(sl[3]));
    ws.vcode[vi] = code;
    // slot of voter i (slots occupy consecutive voter ranges in slot order)
    const int nvote = ws.nvote[b];
    int slot = 0, base = 0, cnt = 0;
    for (int s = 0; s < nvote; s++) {
      const int cls = ws.slot_cls[(size_t)b * C + s];
      base = ws.vbase[(size_t)b * C + cls];
      cnt = ws.vcount[(size_t)b * C + cls];
      slot = s;
      if (i < base + cnt) break;
    }
    const int j = i - base;
    const int y = ws.vpos[vi] / W;
    const int yprev = j > 0 ? ws.vpos[vi - 1] / W : -1;
    int32_t* rs = ws.rowstart + ((size_t)b * C + slot) * (H + 1);
    if (j == 0) {
      rs[y] = 0;
      ws.yspan[((size_t)b * C + slot) * 2] = y;
    } else {
      for (int r = yprev + 1; r <= y; r++) rs[r] = j;  // rows (yprev, y]: usually 0 or 1
    }
    if (j == cnt - 1) ws.yspan[((size_t)b * C + slot) * 2 + 1] = y;
    kslot = slot;
  }
  // slot max of k: lanes grouped by slot (a wave spans at most a few slots),
  // one atomic per (wave, slot) group
  uint64_t active = __ballot(in && k >= 0);
  while (active) {
    const int leader = __ffsll((long long)active) - 1;
    const int s0 = __shfl(kslot, leader, 64);
    const uint64_t m = __ballot(in && k >= 0 && kslot == s0);
    int kk = (in && k >= 0 && kslot == s0) ? k : -1;
    kk = pcnn::wave_max(kk);
    if (pcnn::lane_id() == leader) atomicMax(ws.kmax + (size_t)b * C + s0, kk);
    active &= ~m;
  }
}

}  // namespace pcnn_hough
