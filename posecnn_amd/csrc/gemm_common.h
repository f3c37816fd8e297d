// Shared pieces of the pose-head GEMMs (pose_head.hip: fp32 MFMA and the
// split-bf16 x3 kernel; gemm_x6.hip: the 3-way split-bf16 x6 kernel): the
// argument block, the device-side dims, buffer-descriptor operand views, the
// persistent tile plan and the split-kernel epilogue.
#pragma once
#include "pcnn_common.h"
#include <type_traits>

namespace pcnn_gk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float xf4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  int M, N, K;
  const float* A;
  const float* A2;
  int lda;
  const float* B;
  int ldb;
  float* C;
  int ldc;
  const float* bias;
  int act;
  const float* mask;
  int ldm;
  const int32_t* M_dev;
  const int32_t* K_dev;
  float* slab;  // split-K partials: [kMaxSplit][M][N] (fp32 path), [S][M][N] (split kernels)
  int prec;     // 0 fp32 MFMA, 1 split-bf16 x3, 2 split-bf16 x6 (selects the plan's K step)
  int tile;     // split kernels: tile edge (256 or 128), chosen on the host
  int xgrid;    // split kernels: launch grid (the plan depends on it; k_gemm_reduce re-derives the plan)
  int c_stream; // split kernels: store C non-temporally (outputs far beyond the caches, e.g. the fc6 weight gradient)
  // dropout (pose_head.hip k_gemm_reduce applies it; the GEMM kernels' own
  // epilogues never do): C = (v / keep) * drop[m, n] in the forward; with a
  // mask (the relu + dropout backward) C = (mask > 0 ? v : 0) / keep
  const uint8_t* drop;
  int ldd;
  float keep;  // keep_prob; 1 = no dropout
  // drop_gen: the reduce draws the keep bits itself (Philox, pcnn_philox.h;
  // the same bits pcnn_dropout_mask writes for a dense (M, N) mask) and
  // stores them into drop for the backward
  int drop_gen;
  uint32_t drop_k0, drop_k1, drop_sid;
  const int64_t* drop_step;
};

// The dropout part of the epilogue, after bias / act / mask: tf.nn.dropout's
// (x / keep_prob) * binary (keep == 1: v / 1 == v, the division is skipped).
__device__ __forceinline__ float drop_epi(float v, const GemmArgs& g, int m, int n) {
  if (g.keep != 1.f) v = v / g.keep;
  if (g.drop) v = v * (float)g.drop[(size_t)m * g.ldd + n];
  return v;
}

// Whether the GEMM epilogue of a whole-tile plan already applied 1 / keep
// (x_epilogue, 128-row tiles, no forward drop mask): then k_gemm_reduce has
// nothing left to do for S == 1.
__host__ __device__ __forceinline__ bool keep_in_epilogue(const GemmArgs& g) {
  return g.prec != 0 && g.tile == 128 && g.drop == nullptr;
}

__device__ __forceinline__ int eff_dim(int full, const int32_t* dev) {
  if (!dev) return full;
  int v = *dev;
  return v < full ? (v < 0 ? 0 : v) : full;
}

template <int N>
using IC = std::integral_constant<int, N>;

// K step of a split kernel: 32 (x3: hi / lo planes, 64-B LDS rows) or 16
// (x6: hi / mid / lo planes, 48-B LDS rows; three planes of a 32-deep step
// would not fit two LDS stages)
__host__ __device__ constexpr int split_bk(int prec) { return prec == 2 ? 16 : 32; }

// tile edge of the split kernels for a (capacity) shape
__host__ __device__ __forceinline__ int tile_x3(int M, int N, int K) {
#ifdef PCNN_FORCE_TILE
  return PCNN_FORCE_TILE;
#endif
  return (M <= 128 || N <= 128 || K <= 128) ? 128 : 256;
}

// Plan of the split kernels for an effective shape (M and K may live on the
// device; the host evaluates the same plan for workspace sizing).
//  - M tiles are balanced: mt = ceil(M / T) tiles of Tm rows each, Tm the
//    smallest multiple of 32 >= M / mt (M = 405: 224 + 181 rows, not
//    256 + 149), so the tiles of one N column carry about the same number of
//    live 32-row accumulator blocks; rows past a tile's end are padding whose
//    MFMAs the K loop skips.  The tiles of a column run side by side on one
//    XCD, share their B panel through L2 and finish together (fc6 dX, 196
//    tiles in one round: 318 -> 295 us).
//  - Tile mode: whole tiles dealt round-robin.
//  - Split-K (fewer than G/2 tiles, long K): S K slices per tile, partial
//    slabs reduced in slice order by k_gemm_reduce (the forward shapes); a
//    slice keeps at least 128 of K.
//  Measured and dropped: stream-K over the tiles of a column (K ranges cut
//  evenly over workgroup pairs, partial tiles fixed up in fixed order by the
//  last segment to finish): fc6 dX 295 -> 343 us — the slab round trip and
//  the per-segment fix-up cost more than the balance gains.
#ifndef PCNN_MAX_SPLIT_X
#define PCNN_MAX_SPLIT_X 32
#endif
constexpr int kMaxSplitX = PCNN_MAX_SPLIT_X;  // split-K slices
struct XPlan {
  int mt, nt, ns, Tm, tiles, mode, S;
  bool m_fast;  // tile order: the dimension with fewer tiles runs fastest (its
                // neighbours share the other operand's tile in L2)
  __host__ __device__ int mi_of(int t) const { return m_fast ? t % mt : t / nt; }
  __host__ __device__ int ni_of(int t) const { return m_fast ? t / mt : t % nt; }
};

__host__ __device__ __forceinline__ XPlan x_plan(int Meff, int N, int Keff, int T, int G, int BK) {
  XPlan p;
  p.mt = (Meff + T - 1) / T;
  p.nt = (N + T - 1) / T;
  p.ns = (Keff + BK - 1) / BK;
  p.tiles = p.mt * p.nt;
  p.m_fast = p.mt <= p.nt;
  const int rows = p.mt ? (Meff + p.mt - 1) / p.mt : 0;
  p.Tm = (rows + 31) / 32 * 32;
  p.mode = 0;
  p.S = 1;
#ifdef PCNN_NOSPLIT
  if (false) {
#else
  if (p.tiles > 0 && p.tiles < G / 2) {
#endif
    int s = G / p.tiles;
    if (s > p.ns / (128 / BK)) s = p.ns / (128 / BK);
    if (s > kMaxSplitX) s = kMaxSplitX;
    if (s > 1) {
      p.mode = 1;
      p.S = s;
    }
  }
  return p;
}

// XCD-aware item order: the dispatcher deals workgroup b to XCD b % 8, so a
// bijective remap gives each XCD one contiguous run of items (neighbouring
// tiles share an operand panel through that XCD's L2).  Also for counts that
// are not a multiple of 8 (fc6 dX: 196 tiles, whose two M tiles per N column
// used to land on different XCDs and fetch the same W6 panel twice).
__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n / 8, r = n % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Operand view for buffer loads: SGPR descriptor + the extent in bytes.  All
// per-lane address math is one 32-bit voffset; uniform parts go to soffset.
// Masked lanes use voffset kXOob (>= every extent, < 2^31): the hardware
// range check returns 0 whether or not soffset takes part in it.
constexpr unsigned kXOob = 0x80000000u;
struct XOp {
  __amdgpu_buffer_rsrc_t rs;
  int ld;
  bool valid;
};
__device__ __forceinline__ XOp x_op(const float* P, int ld, long elems) {
  XOp o;
  o.valid = P != nullptr;
  o.rs = __builtin_amdgcn_make_buffer_rsrc((void*)P, (short)0, (int)(elems * 4), 0x00020000);
  o.ld = ld;
  return o;
}
__device__ __forceinline__ float x_ld1(const XOp& o, unsigned voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(o.rs, voff, soff, 0));
}
constexpr int kXNonTemporal = 2;  // buffer cache-policy bit: nt
__device__ __forceinline__ xf4 x_ld4(const XOp& o, unsigned voff, int soff) {
  return __builtin_bit_cast(xf4, __builtin_amdgcn_raw_buffer_load_b128(o.rs, voff, soff, 0));
}

// Exact three-way split of two fp32 values into packed bf16 (hi, mid, lo)
// pairs: one pack-convert per plane; the fp32 value of a packed bf16 half is
// a shift / mask of the pack; both subtractions are exact.  (gemm_x6.hip
// splits while staging; gemm_tp.hip's producer splits once into planes.)
__device__ __forceinline__ void x_split3(float a, float b, unsigned& hi, unsigned& mid, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a, b}, bf16x2));
  const float ra = a - __uint_as_float(hi << 16), rb = b - __uint_as_float(hi & 0xffff0000u);
  mid = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){ra, rb}, bf16x2));
  const float sa = ra - __uint_as_float(mid << 16), sb = rb - __uint_as_float(mid & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){sa, sb}, bf16x2));
}

// Epilogue of one tile (or split-K slice) of a split kernel: AM x AN
// accumulator blocks of 32 x 32 per wave, the wave at rows wm * (T / 2),
// columns wn * 32 AN of the tile.  One uniform branch (slab or C), otherwise
// branch-free: bias / mask come in through buffer loads and results leave
// through buffer stores, out-of-range lanes masked by an out-of-extent offset
// (loads return 0, stores are dropped).  The 16 mask values of group (j, i)
// are issued one group ahead of their use, so the tile pays one mask latency,
// not 8.  Value q of block (i, j) sits at row m0 + rlane + qrow(i, q), column
// n0 + clane + 32 j.  Every per-value term is uniform (a scalar add / compare
// against the lane's one base): left to itself the compiler precomputes a
// lane's 64 row indices once per kernel, spills them, and reloads one per
// store behind a full vmcnt drain.
template <int T, int AM, int AN = 2>
__device__ __forceinline__ void x_epilogue(const GemmArgs& g, const XPlan& pl, const f32x16 (&acc)[AM][AN], int m0,
                                           int n0, int rl, int z, int wm, int wn, int r, int hsel) {
  constexpr int EJ = AN, EI = AM, EQ = 16, EB = 32;
  const int rlane = wm * (T / 2) + 4 * hsel, clane = wn * (32 * AN) + r;
  auto qrow = [](int i, int q) { return i * EB + (q & 3) + 8 * (q >> 2); };
  const int rlim = rl - m0, clim = g.N - n0;  // rows / columns of the tile that exist
  if (pl.mode == 1) {  // split-K slice: raw partial sums to slab z
    const XOp oslab = x_op(g.slab, g.N, (long)pl.S * g.M * g.N);
    const unsigned sb = (unsigned)(((z * g.M + m0 + rlane) * g.N + n0 + clane) * 4);
#pragma unroll
    for (int j = 0; j < EJ; j++)
#pragma unroll
      for (int i = 0; i < EI; i++)
#pragma unroll
        for (int q = 0; q < EQ; q++) {
          const bool ok = clane < clim - j * EB && rlane < rlim - qrow(i, q);
          // (a scalar copy first: __builtin_bit_cast of an ext-vector
          // element subscript reads element 0 with this compiler)
          const float v = acc[i][j][q];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), oslab.rs,
                                                ok ? sb + (unsigned)((qrow(i, q) * g.N + j * EB) * 4) : kXOob,
                                                0, 0);
        }
    return;
  }
  const bool msk = g.mask != nullptr;
  const XOp oc = x_op(g.C, g.ldc, (long)(g.M - 1) * g.ldc + g.N);
  const XOp obias = x_op(g.bias, 0, g.N);
  const XOp omask = x_op(g.mask, g.ldm, g.mask ? (long)(g.M - 1) * g.ldm + g.N : 0);
  const unsigned cbase = (unsigned)(((m0 + rlane) * g.ldc + n0 + clane) * 4);
  const unsigned mbase = (unsigned)(((m0 + rlane) * g.ldm + n0 + clane) * 4);
  float mv[2][EQ];
  auto load_mask = [&](int gi, float (&d)[EQ]) {
    const int j = gi / EI, i = gi % EI;
#pragma unroll
    for (int q = 0; q < EQ; q++) {
      const bool ok = clane < clim - j * EB && rlane < rlim - qrow(i, q);
      d[q] = x_ld1(omask, ok ? mbase + (unsigned)((qrow(i, q) * g.ldm + j * EB) * 4) : kXOob, 0);
    }
  };
  if (msk) load_mask(0, mv[0]);
#pragma unroll
  for (int j = 0; j < EJ; j++) {
    const bool nok = clane < clim - j * EB;
    const float bv = g.bias ? x_ld1(obias, nok ? (unsigned)((n0 + clane + j * EB) * 4) : kXOob, 0) : 0.f;
#pragma unroll
    for (int i = 0; i < EI; i++) {
      const int gi = EI * j + i;
      if (msk && gi + 1 < EJ * EI) load_mask(gi + 1, mv[(gi + 1) & 1]);
#pragma unroll
      for (int q = 0; q < EQ; q++) {
        const bool ok = nok && rlane < rlim - qrow(i, q);
        float v = acc[i][j][q] + bv;
        if (g.act == 1) v = v > 0.f ? v : 0.f;
        if (msk && !(mv[gi & 1][q] > 0.f)) v = 0.f;
        // 128-row tiles: the backward's 1 / keep_prob (no drop mask) applied
        // here rather than by an in-place reduce pass (keep_in_epilogue)
        if constexpr (T == 128)
          if (!g.drop && g.keep != 1.f) v = v / g.keep;
#ifdef PCNN_ABL_NOEPI
        if (v != 1.2345e-30f) continue;
#endif
        const unsigned co = ok ? cbase + (unsigned)((qrow(i, q) * g.ldc + j * EB) * 4) : kXOob;
        if (g.c_stream)  // non-temporal: the output is far larger than L2 + MALL
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), oc.rs, co, 0, kXNonTemporal);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), oc.rs, co, 0, 0);
      }
    }
  }
}

// Launch of the x6 kernel (gemm_x6.hip) for a prepared argument block.
void launch_gemm_x6(const GemmArgs& g, int grid, bool a_trans, bool b_trans, bool ragged, bool a2, bool gen,
                    hipStream_t st);
// LDS bytes of one x6 workgroup at tile edge T
int gemm_x6_lds(int T);

}  // namespace pcnn_gk
