// Pose-head FC contraction for PoseCNN on MI355X (gfx950) — the only MFMA
// user of the hot path.
//
// Replaces the TF matmuls of Network.fc (lib/networks/network.py:393-423) as
// wired by vgg16_convs.py:186-197: pool5 + pool4 -> fc6 (25088 -> 4096, relu)
// -> fc7 (4096 -> 4096, relu) -> fc8 (4096 -> 4C) -> tanh -> * poses_weight ->
// l2_normalize, and their backward products.
//
// GEMM: C = epilogue(op(A) (+ op(A2)) * op(B)) on 128x128 tiles, BK = 16,
// 4 waves per workgroup in a 2x2 arrangement of 64x64 sub-tiles, each a 2x2
// grid of v_mfma_f32_32x32x2_f32 accumulators (exact fp32: the MFMA is an
// fp32 fmaf chain).  The row count M (the RoI rows) and, for the weight
// gradients, the contraction length K may live on the device: the grid is a
// persistent tile loop that reads them, so the whole pose step runs without a
// host sync.  Small-tile-count shapes split K; partial slabs are reduced in
// fixed order by a second kernel that also applies the epilogue (bit-stable
// across runs).  The pool5 + pool4 addition is fused into the A-tile load.
#include "gemm_common.h"
#include "head_common.h"
#include "pcnn_philox.h"
#include <math.h>
#include <stdlib.h>

using namespace pcnn_gk;

namespace {

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int kGemmThreads = 256;
constexpr int kMaxSplit = 8;   // fp32 kernel

// split-K factor for the effective shape (shared by GEMM and reducer)
__host__ __device__ __forceinline__ int split_for(int M, int N, int K) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles >= 256 || M == 0) return 1;
  int s = (512 + tiles - 1) / tiles;
  int smax = K / 512;
  if (s > smax) s = smax;
  if (s > kMaxSplit) s = kMaxSplit;
  return s < 1 ? 1 : s;
}

__device__ __forceinline__ float epilogue(float v, const GemmArgs& g, int m, int n) {
  if (g.bias) v += g.bias[n];
  if (g.act == 1) v = v > 0.f ? v : 0.f;
  if (g.mask && !(g.mask[(size_t)m * g.ldm + n] > 0.f)) v = 0.f;
  return v;
}

// Load a 4-float chunk along the contiguous dimension, zero-filled past `lim`.
__device__ __forceinline__ float4 load4(const float* p, int start, int lim, bool row_ok) {
  if (!row_ok) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (start + 3 < lim && ((((uintptr_t)(p + start)) & 15) == 0)) return *(const float4*)(p + start);
  float4 r;
  r.x = start + 0 < lim ? p[start + 0] : 0.f;
  r.y = start + 1 < lim ? p[start + 1] : 0.f;
  r.z = start + 2 < lim ? p[start + 2] : 0.f;
  r.w = start + 3 < lim ? p[start + 3] : 0.f;
  return r;
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// Tile staging.  A tile is stored in LDS k-major: As[k][m] (m contiguous), the
// layout whose fragment reads (lane: m = l & 31, k = l >> 5) are conflict-free.
template <bool A_T>
struct ATile {
  float4 r[2];
  __device__ __forceinline__ void load(const GemmArgs& g, int m0, int k0, int Meff, int Keff) {
    const int t = threadIdx.x;
    if (!A_T) {  // A (M,K): thread -> row m, two 4-wide k chunks
      const int m = m0 + (t & 127), kq = (t >> 7) * 4;
      const bool ok = m < Meff;
      const float* ar = g.A + (size_t)(ok ? m : 0) * g.lda;
      r[0] = load4(ar, k0 + kq, Keff, ok);
      r[1] = load4(ar, k0 + 8 + kq, Keff, ok);
      if (g.A2) {
        const float* a2 = g.A2 + (size_t)(ok ? m : 0) * g.lda;
        r[0] = add4(r[0], load4(a2, k0 + kq, Keff, ok));
        r[1] = add4(r[1], load4(a2, k0 + 8 + kq, Keff, ok));
      }
    } else {  // A stored (K,M): thread -> k row, 4-wide m chunk
      const int mq = (t & 31) * 4, kr = t >> 5;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = k0 + kr + 8 * h;
        const bool ok = k < Keff;
        const float* ar = g.A + (size_t)(ok ? k : 0) * g.lda;
        r[h] = load4(ar, m0 + mq, Meff, ok);
        if (g.A2) r[h] = add4(r[h], load4(g.A2 + (size_t)(ok ? k : 0) * g.lda, m0 + mq, Meff, ok));
      }
    }
  }
  __device__ __forceinline__ void store(float (*As)[BM]) {
    const int t = threadIdx.x;
    if (!A_T) {
      const int m = t & 127, kq = (t >> 7) * 4;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        As[8 * h + kq + 0][m] = r[h].x;
        As[8 * h + kq + 1][m] = r[h].y;
        As[8 * h + kq + 2][m] = r[h].z;
        As[8 * h + kq + 3][m] = r[h].w;
      }
    } else {
      const int mq = (t & 31) * 4, kr = t >> 5;
#pragma unroll
      for (int h = 0; h < 2; h++) *(float4*)&As[kr + 8 * h][mq] = r[h];
    }
  }
};

template <bool B_T>
struct BTile {
  float4 r[2];
  __device__ __forceinline__ void load(const GemmArgs& g, int n0, int k0, int Keff) {
    const int t = threadIdx.x;
    if (!B_T) {  // B (K,N): thread -> k row, 4-wide n chunk
      const int nq = (t & 31) * 4, kr = t >> 5;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = k0 + kr + 8 * h;
        const bool ok = k < Keff;
        r[h] = load4(g.B + (size_t)(ok ? k : 0) * g.ldb, n0 + nq, g.N, ok);
      }
    } else {  // B stored (N,K): thread -> n row, two 4-wide k chunks
      const int n = n0 + (t & 127), kq = (t >> 7) * 4;
      const bool ok = n < g.N;
      const float* br = g.B + (size_t)(ok ? n : 0) * g.ldb;
      r[0] = load4(br, k0 + kq, Keff, ok);
      r[1] = load4(br, k0 + 8 + kq, Keff, ok);
    }
  }
  __device__ __forceinline__ void store(float (*Bs)[BN]) {
    const int t = threadIdx.x;
    if (!B_T) {
      const int nq = (t & 31) * 4, kr = t >> 5;
#pragma unroll
      for (int h = 0; h < 2; h++) *(float4*)&Bs[kr + 8 * h][nq] = r[h];
    } else {
      const int n = t & 127, kq = (t >> 7) * 4;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        Bs[8 * h + kq + 0][n] = r[h].x;
        Bs[8 * h + kq + 1][n] = r[h].y;
        Bs[8 * h + kq + 2][n] = r[h].z;
        Bs[8 * h + kq + 3][n] = r[h].w;
      }
    }
  }
};

template <bool A_T, bool B_T>
__global__ void __launch_bounds__(kGemmThreads) k_gemm_f32(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[BK][BM];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN];
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  const int mt = (Meff + BM - 1) / BM, nt = (g.N + BN - 1) / BN;
  const int S = split_for(Meff, g.N, Keff);
  const int kchunk = ((Keff + S - 1) / S + BK - 1) / BK * BK;
  const int items = mt * nt * S;
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    // consecutive items share the B (weight) tile: n-tile outermost, m-tile inner
    const int z = item % S;
    const int rest = item / S;
    const int mi = rest % mt, ni = rest / mt;
    const int m0 = mi * BM, n0 = ni * BN;
    const int kb = z * kchunk, ke = min(Keff, kb + kchunk);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = (f32x16){};
    ATile<A_T> at;
    BTile<B_T> bt;
    if (kb < ke) {
      at.load(g, m0, kb, Meff, ke);
      bt.load(g, n0, kb, ke);
    }
    for (int k0 = kb; k0 < ke; k0 += BK) {
      __syncthreads();
      at.store(As);
      bt.store(Bs);
      __syncthreads();
      if (k0 + BK < ke) {  // prefetch the next tile into registers under the MFMAs
        at.load(g, m0, k0 + BK, Meff, ke);
        bt.load(g, n0, k0 + BK, ke);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 2; kk++) {
        const int kr = 2 * kk + (lane >> 5);
        float a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; i++) a[i] = As[kr][wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
        for (int j = 0; j < 2; j++) b[j] = Bs[kr][wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
          for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    // C/D map: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int n = n0 + wn * 64 + j * 32 + (lane & 31);
          if (m < Meff && n < g.N) {
            if (S == 1) g.C[(size_t)m * g.ldc + n] = epilogue(acc[i][j][r], g, m, n);
            else g.slab[((size_t)z * g.M + m) * g.N + n] = acc[i][j][r];
          }
        }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Split-bf16 ("bf16x3") GEMM: x = x_hi + x_lo with x_hi = bf16(x),
// x_lo = bf16(x - x_hi) (16 significant bits), a*b ~ a_hi b_hi + a_hi b_lo +
// a_lo b_hi accumulated in fp32 by v_mfma_f32_32x32x16_bf16 — relative error
// ~1e-5 per product (fp32-class for the 1e-4 quaternion tolerance) at 3/16 of
// the fp32-MFMA cost.  fp32 operands are split while staging into LDS, so the
// weights stay fp32 in HBM (no conversion pass).
//
// Tile 256 x 256 x 32, 512 threads (8 waves as 2 (M) x 4 (N), 128 x 64 per
// wave = 4 x 2 accumulators of 32 x 32), one workgroup per CU with two 64 KiB
// LDS stages: the global loads of step s+2 are in flight (registers) while
// step s computes and step s+1 sits in LDS.  At 512 flop per staged fp32 byte
// pair the tile needs ~21 B/clk/CU at the MFMA rate, inside the L2 share.
// Shapes with an edge <= 128 (the fc8 GEMMs: N = 4C, or K = 4C in dX) use a
// 128 x 128 instance (256 threads, 2 x 2 waves of 64 x 64, two workgroups per
// CU): 4x the workgroups of an output- or latency-bound shape.  Measured
// (scripts/gemm_bench.py): fc8 23-26 us vs 33-40 us at 256; 128 everywhere
// loses 20-25% on fc6 and is even on fc7.
constexpr int XBK = 32;
// Tile geometry: T = 256 (the large shapes) or 128 (shapes with an edge of
// <= 128 or too few 256-tiles to fill the chip: 256 threads as 2 x 2 waves of
// 64 x 64, 64 KiB LDS, two workgroups per CU).
template <int T>
struct XTile {
  static constexpr int threads = 2 * T;
  static constexpr int part = T * 64;       // one operand half (hi or lo): T rows x 32 bf16
  static constexpr int stage = 4 * part;    // a_hi, a_lo, b_hi, b_lo
  static constexpr int lds = 2 * stage;     // 128 / 64 KiB
  static constexpr int grid = T == 256 ? 256 : 512;  // workgroups resident on 256 CUs
  static constexpr int wn = T / 64;         // waves along N (64 columns each); 2 along M
  static constexpr int am = T / 64;         // 32-row accumulators per wave along M
};

// LDS image of an operand half: rows of 64 B = 4 chunks of 8 bf16 (k), chunk
// XOR-swizzled by g(row) = r2 | (r1 ^ r3) << 1 — conflict-free for the
// ds_read_b128 fragment reads (4 x 16-lane groups), the KC-staging
// ds_write_b64 and the NC-staging ds_write_b128 (searched exhaustively over
// linear GF(2) swizzles against the gfx950 lane-group table).
__device__ __forceinline__ int x_off(int row, int c) {
  const int g = ((row >> 2) & 1) | ((((row >> 1) ^ (row >> 3)) & 1) << 1);
  return row * 64 + 16 * (c ^ g);
}

// Staging of one 256-row x 32-k operand tile into 16 fp32 registers.
// KC (operand stored k-contiguous): lane -> k quad t & 7 of rows (t >> 3) + 64 i
// (8 full 128-B lines per load instruction).  NC (stored row-contiguous, k
// rows of ld): wave w takes rows 64 (w >> 1) .. +63 and k 16 (w & 1) .. +15;
// lane l -> row quad l >> 2 (float4 along the row direction) and k quad l & 3,
// so each load instruction reads four 256-B runs and the transposed LDS
// writes of a 16-lane group spread over both halves of each chunk.
// Rows past rlim and k past ke load as 0.  RAGGED: some float4 may straddle
// the K edge (KC) or the row edge (NC) -> element-wise fallback; the common
// instantiation has no divergent branch, so a K step is one basic block.
template <int T, bool KC, bool RAGGED, bool A2>
__device__ __forceinline__ void x_load_part(const XOp& P, const XOp& P2, int r0, int rlim, int k0, int ke,
                                            float (&v)[16], int q) {
  // Every mask is applied to the load ADDRESS (out-of-range voffset -> the
  // hardware returns 0), never to the loaded data: nothing consumes a loaded
  // register before the staging store of the next step, so all loads of a
  // step stay in flight together.  (A2: the summed operand of the generic
  // A + A2 form adds right after its loads.)  Part q = one float4 load.
  const int t = threadIdx.x;
#ifdef PCNN_ABL_L2
  k0 &= 127;  // timing ablation: operands stay L2-resident (wrong results)
#endif
  xf4 x;
  if (KC) {
    const int kq = t & 7;
    const int row = r0 + (t >> 3) + (T / 4) * q;
    const int kl = k0 + 4 * kq;
    const bool ok = row < rlim && kl < ke;
    const unsigned vo = ok ? (unsigned)(row * P.ld + kl) * 4u : kXOob;
    if (!RAGGED || kl + 4 <= ke || !ok) {
      x = x_ld4(P, vo, 0);
      if (A2) x += x_ld4(P2, vo, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const unsigned ve = kl + e < ke ? vo + 4u * e : kXOob;
        x[e] = x_ld1(P, ve, 0);
        if (A2) x[e] += x_ld1(P2, ve, 0);
      }
    }
  } else {
    const int w = t >> 6, l = t & 63;
    const int rq = r0 + 64 * (w >> 1) + 4 * (l >> 2);
    const int k = k0 + 16 * (w & 1) + 4 * (l & 3) + q;
    const bool ok = rq < rlim && k < ke;
    const unsigned vo = ok ? (unsigned)(k * P.ld + rq) * 4u : kXOob;
    if (!RAGGED || rq + 4 <= rlim || !ok) {
      x = x_ld4(P, vo, 0);
      if (A2) x += x_ld4(P2, vo, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const unsigned ve = rq + e < rlim ? vo + 4u * e : kXOob;
        x[e] = x_ld1(P, ve, 0);
        if (A2) x[e] += x_ld1(P2, ve, 0);
      }
    }
  }
  v[4 * q + 0] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
}

template <int T, bool KC, bool RAGGED, bool A2>
__device__ __forceinline__ void x_load(const XOp& P, const XOp& P2, int r0, int rlim, int k0, int ke,
                                       float (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; q++) x_load_part<T, KC, RAGGED, A2>(P, P2, r0, rlim, k0, ke, v, q);
}

// Split of two fp32 values into packed bf16 (hi, lo) pairs: hi = bf16(x)
// (RNE), lo = bf16(x - hi) (the subtraction is exact).  One pack-convert for
// both hi halves, the fp32 value of each hi half by a shift / mask of that
// pack, one pack-convert for both lo halves.
__device__ __forceinline__ void x_split2(float a, float b, unsigned& hi, unsigned& lo) {
#ifdef PCNN_OLDSPLIT
  const __bf16 ha = (__bf16)a, hb = (__bf16)b;
  const __bf16 la = (__bf16)(a - (float)ha), lb = (__bf16)(b - (float)hb);
  hi = (unsigned)__builtin_bit_cast(unsigned short, ha) | ((unsigned)__builtin_bit_cast(unsigned short, hb) << 16);
  lo = (unsigned)__builtin_bit_cast(unsigned short, la) | ((unsigned)__builtin_bit_cast(unsigned short, lb) << 16);
  return;
#endif
  const bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);
  hi = __builtin_bit_cast(unsigned, h);
  const float ah = __uint_as_float(hi << 16), bh = __uint_as_float(hi & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a - ah, b - bh}, bf16x2));
}

// Part q of the split-and-store of a staged operand: KC rows (t >> 3) + T/4 q
// (register quad q); NC row rb + q, i.e. element q of every register quad —
// so an NC part needs all four loads of the operand, a KC part only its own.
template <int T, bool KC>
__device__ __forceinline__ void x_store_part(const float (&v)[16], char* hi, char* lo, int q) {
  const int t = threadIdx.x;
  unsigned h0, h1, l0, l1;
  int o;
  if (KC) {
    const int kq = t & 7;
    const int row = (t >> 3) + (T / 4) * q;
    x_split2(v[4 * q + 0], v[4 * q + 1], h0, l0);
    x_split2(v[4 * q + 2], v[4 * q + 3], h1, l1);
    o = x_off(row, kq >> 1) + (kq & 1) * 8;
  } else {  // v[4 j + e] = (k = k-quad base + j, row = row-quad base + e): transpose into k-contiguous rows
    const int w = t >> 6, l = t & 63;
    const int row = 64 * (w >> 1) + 4 * (l >> 2) + q;
    const int kq = 4 * (w & 1) + (l & 3);  // k quad index 0..7 within the 32-k step
    x_split2(v[q], v[4 + q], h0, l0);
    x_split2(v[8 + q], v[12 + q], h1, l1);
    o = x_off(row, kq >> 1) + (kq & 1) * 8;
  }
  *(uint2*)(hi + o) = make_uint2(h0, h1);
  *(uint2*)(lo + o) = make_uint2(l0, l1);
}

template <int T, bool KC>
__device__ __forceinline__ void x_store(const float (&v)[16], char* hi, char* lo) {
#pragma unroll
  for (int q = 0; q < 4; q++) x_store_part<T, KC>(v, hi, lo, q);
}

// GEN: the general form (split-K and stream-K plans, for device-side M);
// without it the kernel runs whole tiles only (a static-M shape whose plan
// is tile mode, e.g. the weight gradients) and carries none of the partial-
// sum code, which keeps its registers free of spills.
template <int T, bool A_T, bool B_T, bool RAGGED, bool A2, bool GEN>
__global__ void __launch_bounds__(XTile<T>::threads, T == 256 ? 1 : 2) k_gemm_x3(GemmArgs g) {
  using X = XTile<T>;
  constexpr int kXPart = X::part, kXStage = X::stage, AM = X::am;
  extern __shared__ __attribute__((aligned(16))) char xl[];
  constexpr bool A_KC = !A_T, B_KC = B_T;
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  XPlan pl = x_plan(Meff, g.N, Keff, T, g.xgrid, XBK);
  if constexpr (!GEN) {
    pl.mode = 0;
    pl.S = 1;
  }
  const int active = min(g.xgrid, pl.tiles * pl.S);
  // XCD-aware order: the first `active` blocks are dealt round-robin over the
  // 8 XCDs; renumbered so the workgroups of one XCD take consecutive items —
  // the M tiles of a column (one B panel) and neighbouring columns — and
  // shared operand rows meet in one L2
  int wg = blockIdx.x;
  if (wg >= active) return;
#ifndef PCNN_OLD_XCD_MAP
  wg = xcd_remap(wg, active);
#else
  if (active % 8 == 0) wg = (wg % 8) * (active / 8) + wg / 8;
#endif
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  const int wm = wave / X::wn, wn = wave % X::wn;
  const int r = lane & 31, hsel = lane >> 5;
  // operand extents (elements): A (M,K) or (K,M); B (K,N) or (N,K)
  const long a_el = A_T ? (long)(g.K - 1) * g.lda + g.M : (long)(g.M - 1) * g.lda + g.K;
  const long b_el = B_T ? (long)(g.N - 1) * g.ldb + g.K : (long)(g.K - 1) * g.ldb + g.N;
  const XOp oa = x_op(g.A, g.lda, a_el), oa2 = x_op(g.A2, g.lda, a_el), ob = x_op(g.B, g.ldb, b_el),
            onull = x_op(nullptr, 0, 0);
  // fragment offsets (bytes) inside an operand half, per k16 sub-step
  int a_off[2][AM], b_off[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ks++) {
#pragma unroll
    for (int i = 0; i < AM; i++) a_off[ks][i] = x_off(wm * (T / 2) + i * 32 + r, 2 * ks + hsel);
#pragma unroll
    for (int j = 0; j < 2; j++) b_off[ks][j] = x_off(wn * 64 + j * 32 + r, 2 * ks + hsel);
  }

  // One segment: K steps [kl, kh) of tile t, then its epilogue (whole tile)
  // or its slab (+ the fix-up if it is the tile's last segment to finish).
  auto segment = [&](int t, int kl, int kh, int z) {
    const int mi = pl.mi_of(t);
    const int m0 = mi * pl.Tm, n0 = pl.ni_of(t) * T;
    const int rl = min(Meff, m0 + pl.Tm);  // the tile's rows: [m0, rl)
    const int kb = kl * XBK, ke = min(Keff, kh * XBK);
    const int nsteps = kh > kl ? kh - kl : 0;
    // live 32-row accumulator blocks of this wave (rows past the tile are padding)
    const int live = rl - (m0 + wm * (T / 2));
    int amw = live <= 0 ? 0 : (live + 31) / 32;
    amw = __builtin_amdgcn_readfirstlane(amw < AM ? amw : AM);
    f32x16 acc[AM][2];
#pragma unroll
    for (int i = 0; i < AM; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = (f32x16){};
    if (nsteps > 0) {
      float va[16], vb[16];
      // prologue: stage 0 -> LDS buffer 0, stage 1 -> registers
      x_load<T, A_KC, RAGGED, A2>(oa, oa2, m0, rl, kb, ke, va);
      x_load<T, B_KC, RAGGED, false>(ob, onull, n0, g.N, kb, ke, vb);
      x_store<T, A_KC>(va, xl, xl + kXPart);
      x_store<T, B_KC>(vb, xl + 2 * kXPart, xl + 3 * kXPart);
      const int k1 = kb + (nsteps > 1 ? XBK : 0);
      x_load<T, A_KC, RAGGED, A2>(oa, oa2, m0, rl, k1, ke, va);
      x_load<T, B_KC, RAGGED, false>(ob, onull, n0, g.N, k1, ke, vb);
      __syncthreads();
      // Staging part c of step s+1 (registers -> the other LDS buffer) and the
      // matching loads of step s+2 (clamped to the last step: the surplus
      // stores land in a buffer nobody reads).  Parts 0-3 are A, 4-7 B.  The
      // `nxt` buffer was last read in step s-1, before the barrier, so it may
      // be written at any point of step s.
      auto stage_part = [&](int c, char* nxt, int kn) {
        if (c < 4) {
          x_store_part<T, A_KC>(va, nxt, nxt + kXPart, c);
          if (A_KC) {
            x_load_part<T, true, RAGGED, A2>(oa, oa2, m0, rl, kn, ke, va, c);
          } else if (c == 3) {
#pragma unroll
            for (int q = 0; q < 4; q++) x_load_part<T, false, RAGGED, A2>(oa, oa2, m0, rl, kn, ke, va, q);
          }
        } else {
          x_store_part<T, B_KC>(vb, nxt + 2 * kXPart, nxt + 3 * kXPart, c - 4);
          if (B_KC) {
            x_load_part<T, true, RAGGED, false>(ob, onull, n0, g.N, kn, ke, vb, c - 4);
          } else if (c == 7) {
#pragma unroll
            for (int q = 0; q < 4; q++) x_load_part<T, false, RAGGED, false>(ob, onull, n0, g.N, kn, ke, vb, q);
          }
        }
      };
      // The K loop, specialised on AMW = the wave's live accumulator blocks:
      // at M = 405 in 256-row tiles the second tile's lower waves (rows
      // 384-511) have one live block of four, so they issue a quarter of the
      // MFMAs and their SIMD partners run the matrix pipe alone (the schedule
      // weights that tile lighter).  Each specialisation keeps one basic block
      // per K step: after each accumulator row (six MFMAs) its share of the
      // eight staging parts, so the conversion VALU and LDS writes fill MFMA
      // gaps.
      auto kloop = [&](auto amw_c) {
        constexpr int AMW = decltype(amw_c)::value;
        constexpr int SLOTS = 2 * AMW;
        for (int s = 0; s < nsteps; s++) {
          const char* cur = xl + (s & 1) * kXStage;
          char* nxt = xl + ((s + 1) & 1) * kXStage;
          const int kn = kb + (s + 2 < nsteps ? s + 2 : nsteps - 1) * XBK;
          if constexpr (AMW == 0) {
#ifndef PCNN_ABL_NOSTAGE
#pragma unroll
            for (int c = 0; c < 8; c++) stage_part(c, nxt, kn);
#endif
          } else {
#pragma unroll
            for (int ks = 0; ks < 2; ks++) {
              bf16x8 bh[2], bl[2];
#pragma unroll
              for (int j = 0; j < 2; j++) {
                bh[j] = *(const bf16x8*)(cur + 2 * kXPart + b_off[ks][j]);
                bl[j] = *(const bf16x8*)(cur + 3 * kXPart + b_off[ks][j]);
              }
              // A fragments one accumulator row ahead: the reads of row i + 1
              // are in flight while row i's six MFMAs issue
              bf16x8 ah[2], al[2];
              ah[0] = *(const bf16x8*)(cur + a_off[ks][0]);
              al[0] = *(const bf16x8*)(cur + kXPart + a_off[ks][0]);
#pragma unroll
              for (int i = 0; i < AMW; i++) {
                if (i + 1 < AMW) {
                  ah[(i + 1) & 1] = *(const bf16x8*)(cur + a_off[ks][i + 1]);
                  al[(i + 1) & 1] = *(const bf16x8*)(cur + kXPart + a_off[ks][i + 1]);
                }
#pragma unroll
                for (int j = 0; j < 2; j++) {
                  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i & 1], bh[j], acc[i][j], 0, 0, 0);
                  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i & 1], bl[j], acc[i][j], 0, 0, 0);
                  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i & 1], bh[j], acc[i][j], 0, 0, 0);
                }
#ifndef PCNN_ABL_NOSTAGE
                const int slot = ks * AMW + i;
#pragma unroll
                for (int c = slot * 8 / SLOTS; c < (slot + 1) * 8 / SLOTS; c++) stage_part(c, nxt, kn);
#endif
              }
            }
          }
          __syncthreads();
        }
      };
#ifdef PCNN_NOAMW
      kloop(IC<AM>{});
#else
      if (amw == AM) kloop(IC<AM>{});
      else if (amw == 0) kloop(IC<0>{});
      else if (amw == 1) kloop(IC<1>{});
      else if constexpr (AM >= 4) {
        if (amw == 2) kloop(IC<2>{});
        else kloop(IC<3>{});
      }
#endif
    }

    x_epilogue<T, AM>(g, pl, acc, m0, n0, rl, z, wm, wn, r, hsel);
  };

  // this workgroup's items: every active-th (tile, K slice); one call site,
  // so the segment body is instantiated once
  const int kstep = (pl.ns + pl.S - 1) / pl.S;  // split-K: K steps per slice
  for (int item = wg; item < pl.tiles * pl.S; item += active) {
    const int z = item / pl.tiles, t = item % pl.tiles;
    const int kl = z * kstep;
    segment(t, kl, min(pl.ns, kl + kstep), z);
  }
}

// drop_gen: keep byte of element (m, n), drawn (element quad m N/4 + n/4) and
// stored for the backward; the lane whose n is the quad's first stores all four
__device__ __forceinline__ float drop_gen_epi(float v, const GemmArgs& g, uint32_t step, int m, int n) {
  const uint32_t q = pcnn_philox::keep_quad((uint64_t)m * (uint64_t)(g.N >> 2) + (uint64_t)(n >> 2), g.drop_k0,
                                            g.drop_k1, g.drop_sid, step, g.keep);
  if ((n & 3) == 0) *(uint32_t*)((uint8_t*)g.drop + (size_t)m * g.ldd + n) = q;
  if (g.keep != 1.f) v = v / g.keep;
  return v * (float)((q >> (8 * (n & 3))) & 1u);
}

__global__ void __launch_bounds__(256) k_gemm_reduce(GemmArgs g) {
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  const int S = g.prec ? x_plan(Meff, g.N, Keff, g.tile, g.xgrid, split_bk(g.prec)).S : split_for(Meff, g.N, Keff);
  const bool dr = g.drop || g.keep != 1.f;
  const uint32_t step = g.drop_gen && g.drop_step ? (uint32_t)*g.drop_step : 0u;
  auto dropv = [&](float v, int m, int n) { return g.drop_gen ? drop_gen_epi(v, g, step, m, n) : drop_epi(v, g, m, n); };
  if (S == 1) {
    // whole tiles: the GEMM's own epilogue wrote bias / act / mask; dropout
    // (or the backward's 1 / keep) is applied here, in place -- unless the
    // 128-tile epilogue already scaled by 1 / keep
    if (!dr || keep_in_epilogue(g)) return;
    const long total = (long)Meff * g.N;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
      const int m = (int)(i / g.N), n = (int)(i % g.N);
      float* c = g.C + (size_t)m * g.ldc + n;
      *c = dropv(*c, m, n);
    }
    return;
  }
  // slab sums in slice order z = 0, 1, ... (0 + s0 == s0, so starting from
  // s0 is the same fp32 sum); float4 along N when rows stay 16-B aligned
  const size_t slab_stride = (size_t)g.M * g.N;
  const bool vec = (long)g.M * g.N < (1l << 31) && (g.N & 3) == 0 && (g.ldc & 3) == 0 && (!g.mask || (g.ldm & 3) == 0) &&
                   (!g.drop || (g.ldd & 3) == 0) &&
                   ((((uintptr_t)g.slab) | ((uintptr_t)g.C) | ((uintptr_t)g.mask) | ((uintptr_t)g.bias)) & 15) == 0;
  if (vec) {
    const int n4 = g.N >> 2;
    const int total4 = Meff * n4;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
      const int m = i / n4, n = (i - m * n4) << 2;
      const float4* sp = (const float4*)(g.slab + (size_t)m * g.N + n);
      float4 v = sp[0];
      for (int z = 1; z < S; z++) {
        const float4 t = sp[z * (slab_stride >> 2)];
        v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
      }
      float4 o = make_float4(epilogue(v.x, g, m, n), epilogue(v.y, g, m, n + 1), epilogue(v.z, g, m, n + 2),
                             epilogue(v.w, g, m, n + 3));
      if (g.drop_gen) {  // one Philox block per float4: the element quad
        const uint32_t q = pcnn_philox::keep_quad((uint64_t)i, g.drop_k0, g.drop_k1, g.drop_sid, step, g.keep);
        *(uint32_t*)((uint8_t*)g.drop + (size_t)m * g.ldd + n) = q;
        o = make_float4((g.keep != 1.f ? o.x / g.keep : o.x) * (float)(q & 1u),
                        (g.keep != 1.f ? o.y / g.keep : o.y) * (float)((q >> 8) & 1u),
                        (g.keep != 1.f ? o.z / g.keep : o.z) * (float)((q >> 16) & 1u),
                        (g.keep != 1.f ? o.w / g.keep : o.w) * (float)((q >> 24) & 1u));
      } else if (dr) {
        o = make_float4(drop_epi(o.x, g, m, n), drop_epi(o.y, g, m, n + 1), drop_epi(o.z, g, m, n + 2),
                        drop_epi(o.w, g, m, n + 3));
      }
      *(float4*)(g.C + (size_t)m * g.ldc + n) = o;
    }
    return;
  }
  const long total = (long)Meff * g.N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / g.N), n = (int)(i % g.N);
    float v = 0.f;
    for (int z = 0; z < S; z++) v += g.slab[((size_t)z * g.M + m) * g.N + n];
    v = epilogue(v, g, m, n);
    g.C[(size_t)m * g.ldc + n] = dr ? dropv(v, m, n) : v;
  }
}

// Column sums (bias gradients): block = 64 columns x 16 row groups; each thread
// sums rows m = g, g+16, ... (coalesced 256 B rows), the 16 partials are then
// added in fixed order (deterministic).
__global__ void __launch_bounds__(1024) k_colsum(const float* __restrict__ X, int M, int N, int ldx,
                                                 const int32_t* __restrict__ M_dev, float* __restrict__ out) {
  __shared__ float part[16][65];
  const int Meff = eff_dim(M, M_dev);
  const int col = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + col;
  float s = 0.f;
  if (n < N)
    for (int m = grp; m < Meff; m += 16) s += X[(size_t)m * ldx + n];
  part[grp][col] = s;
  __syncthreads();
  if (grp == 0 && n < N) {
    float t = 0.f;
    for (int g = 0; g < 16; g++) t += part[g][col];
    out[n] = t;
  }
}

// one wave per row; D <= 256
__global__ void __launch_bounds__(256) k_head_fwd(const float* __restrict__ y8, const float* __restrict__ pw,
                                                   int R_cap, const int32_t* __restrict__ num_rois_dev, int D,
                                                   float* __restrict__ t_out, float* __restrict__ pred) {
  const int R = eff_dim(R_cap, num_rois_dev);
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = pcnn::lane_id();
  if (row >= R) return;
  float mv[4];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    mv[k] = 0.f;
    if (c < D) {
      const float t = tanhf(y8[(size_t)row * D + c]);
      t_out[(size_t)row * D + c] = t;
      mv[k] = t * pw[(size_t)row * D + c];
      ss += mv[k] * mv[k];
    }
  }
  ss = pcnn::wave_sum(ss);
  const float inv = 1.f / sqrtf(fmaxf(ss, 1e-12f));  // tf.nn.l2_normalize
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    if (c < D) pred[(size_t)row * D + c] = mv[k] * inv;
  }
}

__global__ void __launch_bounds__(256) k_head_bwd(const float* __restrict__ dpred, const float* __restrict__ t_in,
                                                   const float* __restrict__ pw, const float* __restrict__ pred,
                                                   int R_cap, const int32_t* __restrict__ num_rois_dev, int D,
                                                   const float* __restrict__ dscale, float* __restrict__ dy8) {
  const int R = eff_dim(R_cap, num_rois_dev);
  // d_pred = top_diff[0] * bottom_diff when the ADD-loss gradient op is folded
  // in (AveragedistanceBackward, cu.cc:346-354: the same product); 1 * x == x
  const float g = dscale ? dscale[0] : 1.f;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = pcnn::lane_id();
  if (row >= R) return;
  float dp[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    dp[k] = c < D ? g * dpred[(size_t)row * D + c] : 0.f;
  }
  pcnn_head::head_bwd_row(dp, t_in, pw, pred, row, D, lane, dy8);
}

}  // namespace

namespace pcnn_gk {
void launch_gemm_reduce(const GemmArgs& g, hipStream_t st) {
  hipLaunchKernelGGL(k_gemm_reduce, dim3(1024), dim3(256), 0, st, g);
}
}  // namespace pcnn_gk

static int x3_max_grid(int T) { return T == 256 ? XTile<256>::grid : XTile<128>::grid; }

extern "C" size_t pcnn_gemm_workspace_size(int M, int N, int K, int m_dynamic, int precision) {
  if (M <= 0 || N <= 0) return 256;
  if (precision == 1 || precision == 2) {
    // split-K slabs [S][M][N] at the largest split any effective M <= M can take (fewest tiles)
    const int T = tile_x3(M, N, K);
    const XPlan lo = x_plan(m_dynamic ? 1 : M, N, K, T, x3_max_grid(T), split_bk(precision));
    return lo.mode == 1 ? pcnn::align_up((size_t)lo.S * M * N * sizeof(float), 256) + 256 : 256;
  }
  // fp32 path: split-K partial slabs; the split only grows when the device-side M shrinks
  const int s = split_for(m_dynamic ? 1 : M, N, K);
  return s > 1 ? pcnn::align_up((size_t)s * M * N * sizeof(float), 256) + 256 : 256;
}

extern "C" int pcnn_gemm(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B,
                         int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act, const float* mask,
                         int ldm, const int32_t* M_dev, const int32_t* K_dev, int precision, void* workspace,
                         size_t workspace_bytes, void* stream) {
  return pcnn_gemm_drop(M, N, K, A, A2, lda, a_trans, B, ldb, b_trans, Cm, ldc, bias, act, mask, ldm, nullptr, 0, 1.f,
                        M_dev, K_dev, precision, workspace, workspace_bytes, stream);
}

static int gemm_impl(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B,
                     int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act, const float* mask, int ldm,
                     const uint8_t* drop, int ldd, float keep_prob, const int32_t* M_dev, const int32_t* K_dev,
                     int precision, void* workspace, size_t workspace_bytes, void* stream, int drop_gen,
                     uint64_t seed, const int64_t* step_dev, int stream_id) {
  PCNN_REQUIRE(M >= 0 && N > 0 && K >= 0 && A && B && Cm);
  PCNN_REQUIRE(!drop_gen || (drop && N % 4 == 0 && ldd % 4 == 0 && ((uintptr_t)drop & 3) == 0 && stream_id >= 0 &&
                             (long)M * (N / 4) < (1l << 31)));
  PCNN_REQUIRE(keep_prob > 0.f && keep_prob <= 1.f);
  PCNN_REQUIRE(!drop || (ldd >= N && (long)M * ldd < (1l << 31)));
  PCNN_REQUIRE(precision >= 0 && precision <= 2);
  PCNN_REQUIRE(lda >= (a_trans ? M : K) && ldb >= (b_trans ? K : N) && ldc >= N);
  PCNN_REQUIRE(!mask || ldm >= N);
  PCNN_REQUIRE(act == 0 || act == 1);
  // split-bf16 path: 16-B vector staging loads, 32-bit buffer offsets
  PCNN_REQUIRE(precision == 0 || (lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)A & 15) == 0 &&
                                  ((uintptr_t)B & 15) == 0 && (!A2 || ((uintptr_t)A2 & 15) == 0)));
  PCNN_REQUIRE(precision == 0 || ((long)(a_trans ? K : M) * lda < (1l << 29) && (long)(b_trans ? N : K) * ldb < (1l << 29) &&
                                  (long)M * ldc < (1l << 29) && (!mask || (long)M * ldm < (1l << 29))));
  if (M == 0) return PCNN_OK;
  if (workspace_bytes < pcnn_gemm_workspace_size(M, N, K, M_dev != nullptr, precision) || !workspace)
    return PCNN_ECAPACITY;
  GemmArgs g{M, N, K, A, A2, lda, B, ldb, Cm, ldc, bias, act, mask, ldm, M_dev, K_dev, (float*)workspace, precision,
             tile_x3(M, N, K), 0, 0, drop, ldd, keep_prob};
  if (drop_gen) {
    g.drop_gen = 1;
    g.drop_k0 = (uint32_t)seed;
    g.drop_k1 = (uint32_t)(seed >> 32);
    g.drop_sid = (uint32_t)stream_id;
    g.drop_step = step_dev;
  }
  hipStream_t st = (hipStream_t)stream;
  if (precision == 1 || precision == 2) {
    // ragged edges: a KC operand whose K (or device-side K) is not a multiple of
    // 4, or an NC operand whose row count is not -> element-wise edge loads
    const bool a_kc = !a_trans, b_kc = b_trans;
    const bool ragged = ((a_kc || b_kc) && (K % 4 != 0 || K_dev != nullptr)) || (!a_kc && M % 4 != 0) ||
                        (!b_kc && N % 4 != 0);
    const int T = g.tile;
    const int max_grid = x3_max_grid(T);
    long grid = max_grid;
    bool may_split = true, gen = true;
    if (M_dev) {
      // device-side M: the fewest tiles (M = 1) give the largest split; if even
      // that plan runs whole tiles, no effective M splits (fc8 dX, K = 88)
      may_split = x_plan(1, N, K, T, max_grid, split_bk(precision)).mode == 1;
    } else {
      // static M: if the plan runs whole tiles (a device-side K can only lower
      // the split), use the fewest workgroups that keep the same number of
      // rounds (fc6 dW: 1568 tiles -> 224 workgroups x 7): the makespan is
      // unchanged and the spare CUs run the other stream's kernels
      const XPlan pl = x_plan(M, N, K, T, max_grid, split_bk(precision));
      may_split = pl.mode == 1;
      if (pl.mode == 0) {
        gen = T != 256;  // the lean whole-tile kernel (instantiated for T = 256)
        const long items = pl.tiles;
        const long rounds = (items + max_grid - 1) / max_grid;
        grid = (items + rounds - 1) / rounds;
        grid = (grid + 7) / 8 * 8;
        if (grid > max_grid) grid = max_grid;
      }
    }
    g.xgrid = (int)grid;
    // an output larger than the 256 MB MALL is written through without cache
    // allocation (fc6 dW, 411 MB: 316 -> 300 us; the 64 MB fc7 dW and the
    // small activations, re-read by the next GEMM, lose a little with it)
    g.c_stream = (long)M * N * 4 > (256l << 20);
#define PCNN_X3_LAUNCH_G(TT, AT, BT, RG, S2, GN)                                                              \
  do {                                                                                                          \
    static bool attr_set[pcnn::kMaxDevices] = {};                                                               \
    int dev_ = 0;                                                                                               \
    (void)hipGetDevice(&dev_);                                                                                  \
    if (dev_ < 0 || dev_ >= pcnn::kMaxDevices || !attr_set[dev_]) {                                             \
      (void)hipFuncSetAttribute((const void*)k_gemm_x3<TT, AT, BT, RG, S2, GN>,                                 \
                                hipFuncAttributeMaxDynamicSharedMemorySize, XTile<TT>::lds);                    \
      if (dev_ >= 0 && dev_ < pcnn::kMaxDevices) attr_set[dev_] = true;                                         \
    }                                                                                                           \
    hipLaunchKernelGGL((k_gemm_x3<TT, AT, BT, RG, S2, GN>), dim3(grid), dim3(XTile<TT>::threads), XTile<TT>::lds, \
                       st, g);                                                                                  \
  } while (0)
#define PCNN_X3_LAUNCH(AT, BT, RG, S2)                          \
  do {                                                          \
    if (T != 256) PCNN_X3_LAUNCH_G(128, AT, BT, RG, S2, true);  \
    else if (gen) PCNN_X3_LAUNCH_G(256, AT, BT, RG, S2, true);  \
    else PCNN_X3_LAUNCH_G(256, AT, BT, RG, S2, false);          \
  } while (0)
#define PCNN_X3_LAYOUT(RG, S2)                                     \
  do {                                                            \
    if (!a_trans && !b_trans) PCNN_X3_LAUNCH(false, false, RG, S2); \
    else if (!a_trans && b_trans) PCNN_X3_LAUNCH(false, true, RG, S2); \
    else if (a_trans && !b_trans) PCNN_X3_LAUNCH(true, false, RG, S2); \
    else PCNN_X3_LAUNCH(true, true, RG, S2);                       \
  } while (0)
    // split-K slab reduction when the plan can split (a no-op launch is not
    // free: queued behind a persistent GEMM on another stream it holds back
    // everything after it on its own stream); the op's completion event goes
    // to whichever launch is last
    const bool reduce_after = may_split || drop || (keep_prob != 1.f && !keep_in_epilogue(g));
    const hipEvent_t done_ev = reduce_after ? pcnn::take_done_event() : nullptr;
    if (precision == 2) launch_gemm_x6(g, (int)grid, a_trans, b_trans, ragged, A2 != nullptr, gen, st);
    else if (!ragged && !A2) PCNN_X3_LAYOUT(false, false);
    else if (!ragged) PCNN_X3_LAYOUT(false, true);
    else if (!A2) PCNN_X3_LAYOUT(true, false);
    else PCNN_X3_LAYOUT(true, true);
#undef PCNN_X3_LAYOUT
#undef PCNN_X3_LAUNCH_G
#undef PCNN_X3_LAUNCH
    if (reduce_after) {
      pcnn::t_done_event = done_ev;
      pcnn::launch_last(k_gemm_reduce, dim3(1024), dim3(256), 0, st, g);
    }
    PCNN_CHECK_LAUNCH();
    return PCNN_OK;
  }
  const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  // persistent grid sized for the capacity shape at its split
  const long items = (long)mt * nt * split_for(M, N, K);
  long grid = items < 2048 ? items : 2048;
  if (grid < 512) grid = 512;
  if (!a_trans && !b_trans) hipLaunchKernelGGL((k_gemm_f32<false, false>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else if (!a_trans && b_trans) hipLaunchKernelGGL((k_gemm_f32<false, true>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else if (a_trans && !b_trans) hipLaunchKernelGGL((k_gemm_f32<true, false>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else hipLaunchKernelGGL((k_gemm_f32<true, true>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  // split-K slab reduction, unless no device-side M can make the shape split
  // (a static M whose tile count already fills the grid: split 1 for every K).
  // A no-op launch is not free: queued behind a persistent GEMM on another
  // stream it holds back everything after it on its own stream.
  const bool may_split = M_dev || ((M + BM - 1) / BM) * ((N + BN - 1) / BN) < 256 || drop || keep_prob != 1.f;
  if (may_split) hipLaunchKernelGGL(k_gemm_reduce, dim3(1024), dim3(256), 0, st, g);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_gemm_drop(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans,
                              const float* B, int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act,
                              const float* mask, int ldm, const uint8_t* drop, int ldd, float keep_prob,
                              const int32_t* M_dev, const int32_t* K_dev, int precision, void* workspace,
                              size_t workspace_bytes, void* stream) {
  return gemm_impl(M, N, K, A, A2, lda, a_trans, B, ldb, b_trans, Cm, ldc, bias, act, mask, ldm, drop, ldd, keep_prob,
                   M_dev, K_dev, precision, workspace, workspace_bytes, stream, 0, 0, nullptr, 0);
}

extern "C" int pcnn_gemm_drop_gen(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans,
                                  const float* B, int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act,
                                  uint8_t* drop_out, int ldd, float keep_prob, uint64_t seed,
                                  const int64_t* step_dev, int stream_id, const int32_t* M_dev, const int32_t* K_dev,
                                  int precision, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_impl(M, N, K, A, A2, lda, a_trans, B, ldb, b_trans, Cm, ldc, bias, act, nullptr, 0, drop_out, ldd,
                   keep_prob, M_dev, K_dev, precision, workspace, workspace_bytes, stream, 1, seed, step_dev,
                   stream_id);
}

extern "C" int pcnn_colsum(const float* X, int M, int N, int ldx, const int32_t* M_dev, float* out, void* stream) {
  PCNN_REQUIRE(X && out && M >= 0 && N > 0 && ldx >= N);
  hipLaunchKernelGGL(k_colsum, dim3((N + 63) / 64), dim3(1024), 0, (hipStream_t)stream, X, M, N, ldx, M_dev, out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_pose_head_fwd(const float* y8, const float* poses_weight, int R_cap, const int32_t* num_rois_dev,
                                  int D, float* tanh_out, float* pred, void* stream) {
  PCNN_REQUIRE(y8 && poses_weight && tanh_out && pred && R_cap >= 0 && D > 0 && D <= 256);
  if (R_cap == 0) return PCNN_OK;
  hipLaunchKernelGGL(k_head_fwd, dim3((R_cap + 3) / 4), dim3(256), 0, (hipStream_t)stream, y8, poses_weight, R_cap,
                     num_rois_dev, D, tanh_out, pred);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_pose_head_bwd(const float* d_pred, const float* d_pred_scale, const float* tanh_out,
                                  const float* poses_weight, const float* pred, int R_cap,
                                  const int32_t* num_rois_dev, int D, float* d_y8, void* stream) {
  PCNN_REQUIRE(d_pred && tanh_out && poses_weight && pred && d_y8 && R_cap >= 0 && D > 0 && D <= 256);
  if (R_cap == 0) return PCNN_OK;
  hipLaunchKernelGGL(k_head_bwd, dim3((R_cap + 3) / 4), dim3(256), 0, (hipStream_t)stream, d_pred, tanh_out,
                     poses_weight, pred, R_cap, num_rois_dev, D, d_pred_scale, d_y8);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
