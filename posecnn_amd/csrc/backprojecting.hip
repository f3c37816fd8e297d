// Depth backprojection for PoseCNN on MI355X (gfx950).
//
// Replaces BackprojectForwardLaucher / BackprojectBackwardLaucher
// (lib/backprojecting_layer/backprojecting_op_gpu.cu.cc:16-242).
//
// Forward: one thread per (voxel, lane-channel) with the channel innermost, so
// the voxel geometry and the (2k+1)^2 depth tests are wave-uniform and every
// feature read / output write is a coalesced channel sweep.  Label channels are
// handled by lanes c < NC of the same voxel (the reference loops them on the
// c == 0 thread only, cu.cc:62-66, :88-93, which also races with the other
// channel threads' writes of the same voxel); per-channel summation order over
// the neighbourhood (x outer, y inner) is the reference's.
// The output is write-bound: B*G^3*(2Ch+NC)*4 bytes.  These scalar kernels
// serve channel counts that are not multiples of 4; the step's sizes take
// the vector forms below.
#include "pcnn_common.h"
#include <math.h>

namespace {

__global__ void __launch_bounds__(256) k_bp_fwd(const float* __restrict__ data, const float* __restrict__ label,
                                                 const float* __restrict__ depth, const float* __restrict__ meta,
                                                 int num_meta, const float* __restrict__ label_3d, int B, int H, int W,
                                                 int Ch, int NC, int G, int ks, float threshold, int CL,
                                                 float* __restrict__ top_data, float* __restrict__ top_label,
                                                 float* __restrict__ top_flag) {
  const long total = (long)B * G * G * G * CL;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % CL);
    const long vox = idx / CL;
    const int w = (int)(vox % G), h = (int)((vox / G) % G), d = (int)((vox / ((long)G * G)) % G);
    const int n = (int)(vox / ((long)G * G * G));
    const float* m = meta + (size_t)n * num_meta;
    // voxel centre -> live frame -> image (cu.cc:43-60)
    const float X = (float)d * m[42] + m[45];
    const float Y = (float)h * m[43] + m[46];
    const float Z = (float)w * m[44] + m[47];
    const float X1 = m[18] * X + m[19] * Y + m[20] * Z + m[21];
    const float Y1 = m[22] * X + m[23] * Y + m[24] * Z + m[25];
    const float Z1 = m[26] * X + m[27] * Y + m[28] * Z + m[29];
    const float x1 = m[0] * X1 + m[1] * Y1 + m[2] * Z1;
    const float x2 = m[3] * X1 + m[4] * Y1 + m[5] * Z1;
    const float x3 = m[6] * X1 + m[7] * Y1 + m[8] * Z1;
    const int px = (int)roundf(x1 / x3);
    const int py = (int)roundf(x2 / x3);
    const bool do_data = c < Ch, do_label = c < NC;
    float sd = 0.f, sl = 0.f;
    int count = 0;
    for (long x = (long)px - ks; x <= (long)px + ks; x++)
      for (long y = (long)py - ks; y <= (long)py + ks; y++) {
        if (x >= 0 && x < W && y >= 0 && y < H) {
          const size_t ip = ((size_t)n * H + y) * W + x;
          const float dep = depth[ip];
          if (fabsf(dep - Z1) < threshold) {  // cu.cc:79
            count++;
            if (do_data) sd += data[ip * Ch + c];
            if (do_label) sl += label[ip * NC + c];
          }
        }
      }
    if (count == 0) {
      if (do_data) {
        top_data[vox * Ch + c] = 0.f;
        top_flag[vox * Ch + c] = 0.f;
      }
      if (do_label) top_label[vox * NC + c] = label_3d[vox * NC + c];
    } else {
      if (do_data) {
        top_data[vox * Ch + c] = sd / (float)count;
        top_flag[vox * Ch + c] = 1.f;
      }
      if (do_label) top_label[vox * NC + c] = sl / (float)count;
    }
  }
}

__global__ void __launch_bounds__(256) k_bp_bwd(const float* __restrict__ top_diff, const float* __restrict__ depth,
                                                 const float* __restrict__ meta, int num_meta, int B, int H, int W,
                                                 int Ch, int G, float* __restrict__ bottom_diff) {
  const long total = (long)B * H * W * Ch;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % Ch);
    const long pix = idx / Ch;
    const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((long)W * H));
    const float* m = meta + (size_t)n * num_meta;
    const float dep = depth[pix];
    // pixel -> camera ray (Kinv) -> live2world -> voxel (cu.cc:188-210)
    const float RX = m[9] * (float)w + m[10] * (float)h + m[11];
    const float RY = m[12] * (float)w + m[13] * (float)h + m[14];
    const float RZ = m[15] * (float)w + m[16] * (float)h + m[17];
    const float X = dep * RX, Y = dep * RY, Z = dep * RZ;
    const float X1 = m[30] * X + m[31] * Y + m[32] * Z + m[33];
    const float Y1 = m[34] * X + m[35] * Y + m[36] * Z + m[37];
    const float Z1 = m[38] * X + m[39] * Y + m[40] * Z + m[41];
    const int vd = (int)roundf((X1 - m[45]) / m[42]);
    const int vh = (int)roundf((Y1 - m[46]) / m[43]);
    const int vw = (int)roundf((Z1 - m[47]) / m[44]);
    float g = 0.f;
    if (vd >= 0 && vd < G && vh >= 0 && vh < G && vw >= 0 && vw < G)
      g = top_diff[((((size_t)n * G + vd) * G + vh) * G + vw) * Ch + c];
    bottom_diff[idx] = g;
  }
}

// Vector forms (Ch and NC multiples of 4, at most 256), float4 channel
// lanes and 32-bit indexing.  Per channel the neighbourhood sum runs in the
// same (x outer, y inner) order as the scalar kernel, so results are bitwise
// the same.
typedef float f4 __attribute__((ext_vector_type(4)));

// Outputs are stored non-temporally: at the bench size they are 1.2 GB
// (forward) and 629 MB (backward), several times the 256 MB MALL, and are not
// re-read by this op (forward 424 -> 275 us with the channel-lane kernel).
#ifndef PCNN_BP_NT
#define PCNN_BP_NT 1
#endif
__device__ __forceinline__ void bp_st(f4* p, f4 v) {
  if (PCNN_BP_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Runtime kernel size (> 2): a voxel owns LPV lanes, one float4 of channels
// each, so a wave-instruction moves LPV * 16 bytes of one row.
__global__ void __launch_bounds__(256) k_bp_fwd4(const f4* __restrict__ data, const f4* __restrict__ label,
                                                  const float* __restrict__ depth, const float* __restrict__ meta,
                                                  int num_meta, const f4* __restrict__ label_3d, int B, int H, int W,
                                                  int Ch4, int NC4, int G, int ks_rt, float threshold, int lpv_log2,
                                                  f4* __restrict__ top_data, f4* __restrict__ top_label,
                                                  f4* __restrict__ top_flag) {
  const int ks = ks_rt;
  const int lane = threadIdx.x & 63;
  const int sub = lane >> lpv_log2, cq = lane & ((1 << lpv_log2) - 1);
  const int vpw = 64 >> lpv_log2;
  const int GG = G * G, G3 = GG * G, nvox = B * G3;
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (int v0 = wv * vpw; v0 < nvox; v0 += nw * vpw) {
    const int vox = v0 + sub;
    if (vox >= nvox) continue;
    const int n = vox / G3, r3 = vox - n * G3, d = r3 / GG, r2 = r3 - d * GG, h = r2 / G, w = r2 - h * G;
    const float* m = meta + (size_t)n * num_meta;
    // voxel centre -> live frame -> image (cu.cc:43-60)
    const float X = (float)d * m[42] + m[45];
    const float Y = (float)h * m[43] + m[46];
    const float Z = (float)w * m[44] + m[47];
    const float X1 = m[18] * X + m[19] * Y + m[20] * Z + m[21];
    const float Y1 = m[22] * X + m[23] * Y + m[24] * Z + m[25];
    const float Z1 = m[26] * X + m[27] * Y + m[28] * Z + m[29];
    const float x1 = m[0] * X1 + m[1] * Y1 + m[2] * Z1;
    const float x2 = m[3] * X1 + m[4] * Y1 + m[5] * Z1;
    const float x3 = m[6] * X1 + m[7] * Y1 + m[8] * Z1;
    const int px = (int)roundf(x1 / x3);
    const int py = (int)roundf(x2 / x3);
    const bool do_data = cq < Ch4, do_label = cq < NC4;
    f4 sd = {0.f, 0.f, 0.f, 0.f}, sl = {0.f, 0.f, 0.f, 0.f};
    int count = 0;
    auto visit = [&](int x, int y, bool hit) {
      if (hit) {
        const int ip = (n * H + y) * W + x;
        count++;
        if (do_data) sd += data[(size_t)ip * Ch4 + cq];
        if (do_label) sl += label[(size_t)ip * NC4 + cq];
      }
    };
    for (int x = px - ks; x <= px + ks; x++)
      for (int y = py - ks; y <= py + ks; y++) {
        const bool in = x >= 0 && x < W && y >= 0 && y < H;
        visit(x, y, in && fabsf(depth[in ? (n * H + y) * W + x : 0] - Z1) < threshold);  // cu.cc:79
      }
    if (do_data) {
      const float cf = (float)count;
      bp_st(top_data + (size_t)vox * Ch4 + cq, count ? sd / cf : (f4){0.f, 0.f, 0.f, 0.f});
      const float fl = count ? 1.f : 0.f;
      bp_st(top_flag + (size_t)vox * Ch4 + cq, (f4){fl, fl, fl, fl});
    }
    if (do_label)
      bp_st(top_label + (size_t)vox * NC4 + cq,
            count ? sl / (float)count : label_3d[(size_t)vox * NC4 + cq]);
  }
}

// Compile-time neighbourhood (KS = 0, 1, 2), 64 voxels per wave pass.
// Phase 1: lane l owns voxel v0 + l and does its geometry and its (2KS+1)^2
// depth tests once (the channel-lane form repeats them on every channel lane
// of a voxel, and that VALU work, not HBM, set its time).  Phase 2: the pass's
// outputs are contiguous runs (64 * Ch4 float4 of top_data / top_flag,
// 64 * NC4 of top_label), so lane l writes float4 l + 64 k of each run, a full
// 1 KiB per store instruction.  The element's voxel (e / Ch4, exact by a
// 2^20 fixed-point reciprocal for e < 4096) fetches its hit mask from the
// owning lane; only voxels with hits gather feature rows, in the reference's
// (x outer, y inner) order.
template <int KS>
__global__ void __launch_bounds__(256) k_bp_fwd4w(const f4* __restrict__ data, const f4* __restrict__ label,
                                                   const float* __restrict__ depth, const float* __restrict__ meta,
                                                   int num_meta, const f4* __restrict__ label_3d, int B, int H, int W,
                                                   int Ch4, int NC4, int G, float threshold, unsigned rcp_ch4,
                                                   unsigned rcp_nc4, f4* __restrict__ top_data,
                                                   f4* __restrict__ top_label, f4* __restrict__ top_flag) {
  constexpr int S = 2 * KS + 1;
  const int lane = threadIdx.x & 63;
  const int GG = G * G, G3 = GG * G, nvox = B * G3;
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (int v0 = wv * 64; v0 < nvox; v0 += nw * 64) {
    // phase 1: one voxel per lane
    const int vox = min(v0 + lane, nvox - 1);
    const int n = vox / G3, r3 = vox - n * G3, d = r3 / GG, r2 = r3 - d * GG, h = r2 / G, w = r2 - h * G;
    const float* m = meta + (size_t)n * num_meta;
    // voxel centre -> live frame -> image (cu.cc:43-60)
    const float X = (float)d * m[42] + m[45];
    const float Y = (float)h * m[43] + m[46];
    const float Z = (float)w * m[44] + m[47];
    const float X1 = m[18] * X + m[19] * Y + m[20] * Z + m[21];
    const float Y1 = m[22] * X + m[23] * Y + m[24] * Z + m[25];
    const float Z1 = m[26] * X + m[27] * Y + m[28] * Z + m[29];
    const float x1 = m[0] * X1 + m[1] * Y1 + m[2] * Z1;
    const float x2 = m[3] * X1 + m[4] * Y1 + m[5] * Z1;
    const float x3 = m[6] * X1 + m[7] * Y1 + m[8] * Z1;
    const int px = (int)roundf(x1 / x3);
    const int py = (int)roundf(x2 / x3);
    unsigned mask = 0;
#pragma unroll
    for (int i = 0; i < S * S; i++) {  // bit i: neighbour (x = px - KS + i / S, y = py - KS + i % S)
      const int x = px - KS + i / S, y = py - KS + i % S;
      const bool in = x >= 0 && x < W && y >= 0 && y < H;
      const float dep = depth[in ? (n * H + y) * W + x : 0];
      mask |= (in && fabsf(dep - Z1) < threshold) ? (1u << i) : 0u;  // cu.cc:79
    }
    const int nv = min(64, nvox - v0);
    const bool any = __ballot(mask != 0 && lane < nv) != 0;
    // the hit path needs the owner's pixel base: (n * H + py - KS) * W + px - KS
    const int base = (n * H + py - KS) * W + px - KS;

    // phase 2: contiguous output runs of this pass
    auto fetch = [&](int e, unsigned rcp, int& vi, unsigned& mk, int& bs) {
      vi = (int)(((unsigned)e * rcp) >> 20);
      mk = (unsigned)__shfl((int)mask, vi);
      bs = any ? __shfl(base, vi) : 0;
    };
    for (int k = 0; k < Ch4; k++) {
      const int e = lane + 64 * k;
      int vi, bs;
      unsigned mk;
      fetch(e, rcp_ch4, vi, mk, bs);
      if (vi >= nv) continue;
      const int cq = e - vi * Ch4;
      f4 sd = {0.f, 0.f, 0.f, 0.f};
      int count = 0;
      if (mk) {
#pragma unroll
        for (int i = 0; i < S * S; i++)  // x outer, y inner
          if (mk & (1u << i)) {
            count++;
            sd += data[(size_t)(bs + (i % S) * W + i / S) * Ch4 + cq];
          }
      }
      const float fl = count ? 1.f : 0.f;
      bp_st(top_data + (size_t)v0 * Ch4 + e, count ? sd / (float)count : (f4){0.f, 0.f, 0.f, 0.f});
      bp_st(top_flag + (size_t)v0 * Ch4 + e, (f4){fl, fl, fl, fl});
    }
    for (int k = 0; k < NC4; k++) {
      const int e = lane + 64 * k;
      int vi, bs;
      unsigned mk;
      fetch(e, rcp_nc4, vi, mk, bs);
      if (vi >= nv) continue;
      const int cq = e - vi * NC4;
      if (!mk) {
        bp_st(top_label + (size_t)v0 * NC4 + e, label_3d[(size_t)v0 * NC4 + e]);
        continue;
      }
      f4 sl = {0.f, 0.f, 0.f, 0.f};
      int count = 0;
#pragma unroll
      for (int i = 0; i < S * S; i++)
        if (mk & (1u << i)) {
          count++;
          sl += label[(size_t)(bs + (i % S) * W + i / S) * NC4 + cq];
        }
      bp_st(top_label + (size_t)v0 * NC4 + e, sl / (float)count);
    }
  }
}

// Backward with one pixel per lane for the geometry (64 pixels a wave pass),
// then the pass's 64 * Ch4 float4 of bottom_diff written as contiguous 1 KiB
// store instructions; element e belongs to pixel e / Ch4 and reads that
// pixel's top_diff row (or writes zero outside the grid).
__global__ void __launch_bounds__(256) k_bp_bwd4w(const f4* __restrict__ top_diff, const float* __restrict__ depth,
                                                   const float* __restrict__ meta, int num_meta, int B, int H, int W,
                                                   int Ch4, int G, unsigned rcp_ch4, f4* __restrict__ bottom_diff) {
  const int lane = threadIdx.x & 63;
  const int HW = H * W, npix = B * HW;
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (int p0 = wv * 64; p0 < npix; p0 += nw * 64) {
    const int pix = min(p0 + lane, npix - 1);
    const int n = pix / HW, r = pix - n * HW, h = r / W, w = r - h * W;
    const float* m = meta + (size_t)n * num_meta;
    const float dep = depth[pix];
    // pixel -> camera ray (Kinv) -> live2world -> voxel (cu.cc:188-210)
    const float RX = m[9] * (float)w + m[10] * (float)h + m[11];
    const float RY = m[12] * (float)w + m[13] * (float)h + m[14];
    const float RZ = m[15] * (float)w + m[16] * (float)h + m[17];
    const float X = dep * RX, Y = dep * RY, Z = dep * RZ;
    const float X1 = m[30] * X + m[31] * Y + m[32] * Z + m[33];
    const float Y1 = m[34] * X + m[35] * Y + m[36] * Z + m[37];
    const float Z1 = m[38] * X + m[39] * Y + m[40] * Z + m[41];
    const int vd = (int)roundf((X1 - m[45]) / m[42]);
    const int vh = (int)roundf((Y1 - m[46]) / m[43]);
    const int vw = (int)roundf((Z1 - m[47]) / m[44]);
    const int row = (vd >= 0 && vd < G && vh >= 0 && vh < G && vw >= 0 && vw < G) ? ((n * G + vd) * G + vh) * G + vw
                                                                                   : -1;
    const int np = min(64, npix - p0);
    for (int k = 0; k < Ch4; k++) {
      const int e = lane + 64 * k;
      const int pi = (int)(((unsigned)e * rcp_ch4) >> 20);
      const int rw = __shfl(row, pi);
      if (pi >= np) continue;
      const f4 g = rw >= 0 ? top_diff[(size_t)rw * Ch4 + (e - pi * Ch4)] : (f4){0.f, 0.f, 0.f, 0.f};
      bp_st(bottom_diff + (size_t)p0 * Ch4 + e, g);
    }
  }
}

static int lpv_log2_for(int c4) {  // lanes per row: the smallest power of two >= c4 (c4 <= 64)
  int l = 0;
  while ((1 << l) < c4) l++;
  return l;
}
static bool bp_vec_ok(const void* a, const void* b, int ch) {
  return ch % 4 == 0 && ch <= 256 && ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
}

}  // namespace

extern "C" int pcnn_backproject_fwd(const float* data, const float* label, const float* depth, const float* meta,
                                    int num_meta, const float* label_3d, int B, int H, int W, int Ch, int NC,
                                    int grid_size, int kernel_size, float threshold, float* top_data,
                                    float* top_label, float* top_flag, void* stream) {
  PCNN_REQUIRE(data && label && depth && meta && label_3d && top_data && top_label && top_flag);
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && Ch > 0 && NC > 0 && grid_size > 0 && kernel_size >= 0 && num_meta >= 48);
  const int CL = Ch > NC ? Ch : NC;
  const long nvox = (long)B * grid_size * grid_size * grid_size;
  if (bp_vec_ok(data, top_data, Ch) && bp_vec_ok(label, top_label, NC) && bp_vec_ok(label_3d, top_flag, NC) &&
      nvox * (CL / 4) < (1l << 31) && (long)B * H * W < (1l << 31)) {
    const int lg = lpv_log2_for(CL / 4);
    const long waves = (nvox + (64 >> lg) - 1) / (64 >> lg);
    const long bcap = 65536;
    const long wu = kernel_size <= 2 ? (nvox + 63) / 64 : waves;  // k_bp_fwd4w: 64 voxels a wave pass
    const int blocks = (int)((wu + 3) / 4 < bcap ? (wu + 3) / 4 : bcap);
    const unsigned rcp_ch4 = ((1u << 20) + Ch / 4 - 1) / (Ch / 4), rcp_nc4 = ((1u << 20) + NC / 4 - 1) / (NC / 4);
#define PCNN_BP_FWD4(KS)                                                                                     \
  hipLaunchKernelGGL(k_bp_fwd4, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const f4*)data,            \
                     (const f4*)label, depth, meta, num_meta, (const f4*)label_3d, B, H, W, Ch / 4, NC / 4,      \
                     grid_size, kernel_size, threshold, lg, (f4*)top_data, (f4*)top_label, (f4*)top_flag)
#define PCNN_BP_FWD4U(KS)                                                                                    \
  hipLaunchKernelGGL((k_bp_fwd4w<KS>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const f4*)data,        \
                     (const f4*)label, depth, meta, num_meta, (const f4*)label_3d, B, H, W, Ch / 4, NC / 4,      \
                     grid_size, threshold, rcp_ch4, rcp_nc4, (f4*)top_data, (f4*)top_label, (f4*)top_flag)
    if (kernel_size == 0) PCNN_BP_FWD4U(0);
    else if (kernel_size == 1) PCNN_BP_FWD4U(1);
    else if (kernel_size == 2) PCNN_BP_FWD4U(2);
    else PCNN_BP_FWD4();
#undef PCNN_BP_FWD4
    PCNN_CHECK_LAUNCH();
    return PCNN_OK;
  }
  const long total = nvox * CL;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(k_bp_fwd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, data, label, depth, meta, num_meta,
                     label_3d, B, H, W, Ch, NC, grid_size, kernel_size, threshold, CL, top_data, top_label, top_flag);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_backproject_bwd(const float* top_diff, const float* depth, const float* meta, int num_meta, int B,
                                    int H, int W, int Ch, int grid_size, float* bottom_diff, void* stream) {
  PCNN_REQUIRE(top_diff && depth && meta && bottom_diff && B > 0 && H > 0 && W > 0 && Ch > 0 && grid_size > 0);
  PCNN_REQUIRE(num_meta >= 48);
  const long npix = (long)B * H * W;
  if (bp_vec_ok(top_diff, bottom_diff, Ch) && npix * (Ch / 4) < (1l << 31)) {
    const long waves = (npix + 63) / 64;
    const int blocks = (int)((waves + 3) / 4 < 65536 ? (waves + 3) / 4 : 65536);
    const unsigned rcp_ch4 = ((1u << 20) + Ch / 4 - 1) / (Ch / 4);
    hipLaunchKernelGGL(k_bp_bwd4w, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const f4*)top_diff, depth, meta,
                       num_meta, B, H, W, Ch / 4, grid_size, rcp_ch4, (f4*)bottom_diff);
    PCNN_CHECK_LAUNCH();
    return PCNN_OK;
  }
  const long total = npix * Ch;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(k_bp_bwd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, top_diff, depth, meta, num_meta, B,
                     H, W, Ch, grid_size, bottom_diff);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
