// Three-way split-bf16 ("bf16x6") GEMM for the pose-head FC layers — the
// fp32-faithful MFMA path (precision 2) of pcnn_gemm (pose_head.hip).
//
// The reference runs fc6 / fc7 / fc8 as fp32 tf.matmul
// (lib/networks/network.py:393-423, wired at vgg16_convs.py:186-197).  Every
// fp32 x splits EXACTLY into three bf16 planes: hi = bf16(x), mid =
// bf16(x - hi), lo = x - hi - mid (x - hi has at most 16 significant bits, so
// x - hi - mid has at most 8 and is a bf16; both subtractions are exact).
// a*b = sum of the nine plane products; the six kept here (hi*hi, hi*mid,
// mid*hi, mid*mid, hi*lo, lo*hi) leave out mid*lo + lo*mid + lo*lo, below
// 2^-24 |a||b| -- under fp32's own rounding of the product.  Each bf16 x bf16
// product is exact in fp32 and v_mfma_f32_32x32x16_bf16 accumulates in fp32,
// so a K-term dot product carries fp32 accumulation error with six roundings
// per 16 terms where an fmaf chain has sixteen: the same error class as the
// reference's fp32 GEMM, at 6/16 of the fp32-MFMA cost (bf16 MFMA issues 16x
// the flops of v_mfma_f32_32x32x2_f32 per cycle).
//
// Structure as k_gemm_x3 (pose_head.hip): a persistent tile loop over a
// device-side plan (balanced M tiles, split-K slabs for the forward shapes,
// XCD-aware item order), fp32 operands split while staging into LDS (the
// weights stay fp32 in HBM), two LDS stages with the loads of step s+2 in
// registers, the staging parts interleaved with the MFMA rows, and the K loop
// specialised on the wave's live accumulator blocks.  Differences: the K step
// is 16 (three planes of a 32-deep step would need 192 KiB for two stages),
// and an LDS plane row is 48 B (16 bf16 + 16 B of padding): with 12-word rows
// the ds_read_b128 fragment reads, the k-contiguous ds_write_b64 staging and
// the transposing ds_write_b32 staging of row-contiguous operands are all
// conflict-free or 2-way (free for b32 writes) without an XOR swizzle, which a
// 2-chunk row cannot provide.  Tile 256: 6 planes x 12 KiB = 72 KiB per stage,
// 144 KiB for two, one workgroup per CU; tile 128: 72 KiB, two per CU.
#include "gemm_common.h"

using namespace pcnn_gk;

namespace {

constexpr int X6BK = 16;
constexpr int kRow = 48;  // bytes per LDS plane row

template <int T>
struct X6Tile {
  static constexpr int threads = 2 * T;
  static constexpr int part = T * kRow;   // one plane of one operand: T rows x 16 bf16 (+ pad)
  static constexpr int stage = 6 * part;  // a_hi, a_mid, a_lo, b_hi, b_mid, b_lo
  static constexpr int lds = 2 * stage;   // 144 / 72 KiB
  static constexpr int wn = T / 64;       // waves along N (64 columns each); 2 along M
  static constexpr int am = T / 64;       // 32-row accumulators per wave along M
};

__device__ __forceinline__ int x6_off(int row, int c) { return row * kRow + 16 * c; }

// k-contiguous staging: lane t -> k quad t & 3 of row x6_kc_row(t) + (T/2) q.
// A 16-lane write group covers rows {0, 2, 4, 6} or {1, 3, 5, 7} (+ 8 n): at
// 12 words per row their 8-word spans tile the 32 banks exactly.
__device__ __forceinline__ int x6_kc_row(int t) { return 8 * (t >> 5) + 2 * ((t >> 2) & 3) + ((t >> 4) & 1); }

// Staging of one T-row x 16-k operand tile into 8 fp32 registers (two float4
// loads, part q = load q).  KC: rows x6_kc_row(t) + (T/2) q, k quad t & 3 (a
// wave reads 16 row segments of 64 B).  NC (stored row-contiguous, k rows of
// ld): lane t -> row quad t >> 3 (float4 along the rows) at k = 2 (t & 7) + q,
// so a wave reads 8 k rows x 128 B.  Masks go to the load address (the
// hardware returns 0 past the extent); RAGGED: a float4 may straddle the K
// edge (KC) or the row edge (NC) -> element-wise.
template <int T, bool KC, bool RAGGED, bool A2>
__device__ __forceinline__ void x6_load_part(const XOp& P, const XOp& P2, int r0, int rlim, int k0, int ke,
                                             float (&v)[8], int q) {
  const int t = threadIdx.x;
  xf4 x;
  if (KC) {
    const int kq = t & 3;
    const int row = r0 + x6_kc_row(t) + (T / 2) * q;
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
    const int rq = r0 + 4 * (t >> 3);
    const int k = k0 + 2 * (t & 7) + q;
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

// Part q of the split-and-store of a staged operand into its three planes
// (pl, pl + part, pl + 2 part).  KC: row x6_kc_row(t) + (T/2) q, 4 k -> one
// ds_write_b64 per plane.  NC: rows 4 (t >> 3) + 2q + {0, 1}, the k pair
// 2 (t & 7) + {0, 1} from loads 0 and 1 -> one ds_write_b32 per row and plane
// (so an NC part needs both loads of the operand).
template <int T, bool KC>
__device__ __forceinline__ void x6_store_part(const float (&v)[8], char* pl, int q) {
  constexpr int P = X6Tile<T>::part;
  const int t = threadIdx.x;
  if (KC) {
    unsigned h0, m0, l0, h1, m1, l1;
    x_split3(v[4 * q + 0], v[4 * q + 1], h0, m0, l0);
    x_split3(v[4 * q + 2], v[4 * q + 3], h1, m1, l1);
    const int o = (x6_kc_row(t) + (T / 2) * q) * kRow + 8 * (t & 3);
    *(uint2*)(pl + o) = make_uint2(h0, h1);
    *(uint2*)(pl + P + o) = make_uint2(m0, m1);
    *(uint2*)(pl + 2 * P + o) = make_uint2(l0, l1);
  } else {
#pragma unroll
    for (int d = 0; d < 2; d++) {
      const int e = 2 * q + d;
      unsigned h, m, l;
      x_split3(v[e], v[4 + e], h, m, l);
      const int o = (4 * (t >> 3) + e) * kRow + 4 * (t & 7);
      *(unsigned*)(pl + o) = h;
      *(unsigned*)(pl + P + o) = m;
      *(unsigned*)(pl + 2 * P + o) = l;
    }
  }
}

#ifdef PCNN_X6_NOREAD  // timing ablation (wrong results): fragments from a register, no LDS reads
#define X6_FRAG(ptr) (fake)
#else
#define X6_FRAG(ptr) (*(const bf16x8*)(ptr))
#endif

template <int T, bool A_T, bool B_T, bool RAGGED, bool A2, bool GEN>
__global__ void __launch_bounds__(X6Tile<T>::threads, T == 256 ? 1 : 2) k_gemm_x6(GemmArgs g) {
  using X = X6Tile<T>;
  constexpr int PART = X::part, STAGE = X::stage, AM = X::am;
  extern __shared__ __attribute__((aligned(16))) char xl[];
  constexpr bool A_KC = !A_T, B_KC = B_T;
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  XPlan pl = x_plan(Meff, g.N, Keff, T, g.xgrid, X6BK);
  if constexpr (!GEN) {
    pl.mode = 0;
    pl.S = 1;
  }
  const int active = min(g.xgrid, pl.tiles * pl.S);
  // XCD-aware order (as k_gemm_x3): the workgroups of one XCD take consecutive items
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
#ifdef PCNN_X6_NOREAD
  bf16x8 fake;
  for (int e = 0; e < 8; e++) fake[e] = (__bf16)(float)((lane * 7 + e) & 15);
#endif
  const long a_el = A_T ? (long)(g.K - 1) * g.lda + g.M : (long)(g.M - 1) * g.lda + g.K;
  const long b_el = B_T ? (long)(g.N - 1) * g.ldb + g.K : (long)(g.K - 1) * g.ldb + g.N;
  const XOp oa = x_op(g.A, g.lda, a_el), oa2 = x_op(g.A2, g.lda, a_el), ob = x_op(g.B, g.ldb, b_el),
            onull = x_op(nullptr, 0, 0);
  // fragment offsets (bytes) inside a plane: lane -> row r, k 8 hsel .. +7
  int a_off[AM], b_off[2];
#pragma unroll
  for (int i = 0; i < AM; i++) a_off[i] = x6_off(wm * (T / 2) + i * 32 + r, hsel);
#pragma unroll
  for (int j = 0; j < 2; j++) b_off[j] = x6_off(wn * 64 + j * 32 + r, hsel);

  auto segment = [&](int t, int kl, int kh, int z) {
    const int m0 = pl.mi_of(t) * pl.Tm, n0 = pl.ni_of(t) * T;
    const int rl = min(Meff, m0 + pl.Tm);
    const int kb = kl * X6BK, ke = min(Keff, kh * X6BK);
    const int nsteps = kh > kl ? kh - kl : 0;
    const int live = rl - (m0 + wm * (T / 2));
    int amw = live <= 0 ? 0 : (live + 31) / 32;
    amw = __builtin_amdgcn_readfirstlane(amw < AM ? amw : AM);
    f32x16 acc[AM][2];
#pragma unroll
    for (int i = 0; i < AM; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = (f32x16){};
#ifdef PCNN_X6_M16ABL
    f32x4 a16[AM][2][4];
#pragma unroll
    for (int i = 0; i < AM; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int p = 0; p < 4; p++) a16[i][j][p] = (f32x4){};
#endif
    if (nsteps > 0) {
      float va[8], vb[8];
      // prologue: stage 0 -> LDS buffer 0, stage 1 -> registers
#pragma unroll
      for (int q = 0; q < 2; q++) {
        x6_load_part<T, A_KC, RAGGED, A2>(oa, oa2, m0, rl, kb, ke, va, q);
        x6_load_part<T, B_KC, RAGGED, false>(ob, onull, n0, g.N, kb, ke, vb, q);
      }
#pragma unroll
      for (int q = 0; q < 2; q++) {
        x6_store_part<T, A_KC>(va, xl, q);
        x6_store_part<T, B_KC>(vb, xl + 3 * PART, q);
      }
      const int k1 = kb + (nsteps > 1 ? X6BK : 0);
#pragma unroll
      for (int q = 0; q < 2; q++) {
        x6_load_part<T, A_KC, RAGGED, A2>(oa, oa2, m0, rl, k1, ke, va, q);
        x6_load_part<T, B_KC, RAGGED, false>(ob, onull, n0, g.N, k1, ke, vb, q);
      }
      __syncthreads();
      // staging part c of step s+1 (registers -> the other LDS buffer) and the
      // matching load of step s+2 (clamped to the last step: surplus stores
      // land in a buffer nobody reads); parts 0-1 are A, 2-3 B
      auto stage_part = [&](int c, char* nxt, int kn) {
        if (c < 2) {
          x6_store_part<T, A_KC>(va, nxt, c);
          if (A_KC) {
            x6_load_part<T, true, RAGGED, A2>(oa, oa2, m0, rl, kn, ke, va, c);
          } else if (c == 1) {
#pragma unroll
            for (int q = 0; q < 2; q++) x6_load_part<T, false, RAGGED, A2>(oa, oa2, m0, rl, kn, ke, va, q);
          }
        } else {
          x6_store_part<T, B_KC>(vb, nxt + 3 * PART, c - 2);
          if (B_KC) {
            x6_load_part<T, true, RAGGED, false>(ob, onull, n0, g.N, kn, ke, vb, c - 2);
          } else if (c == 3) {
#pragma unroll
            for (int q = 0; q < 2; q++) x6_load_part<T, false, RAGGED, false>(ob, onull, n0, g.N, kn, ke, vb, q);
          }
        }
      };
      // K loop specialised on the wave's live accumulator blocks (AMW); each
      // step is one basic block: per accumulator row twelve MFMAs, then its
      // share of the four staging parts.  Products are accumulated smallest
      // first (lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi).
      auto kloop = [&](auto amw_c, auto first_c) {
        constexpr int AMW = decltype(amw_c)::value;
        // 0: each row's staging share after its MFMAs; 1: before them;
        // 2: all staging before the rows; 3: all staging after the rows
        constexpr int MODE = decltype(first_c)::value;
        constexpr bool STAGE_FIRST = MODE == 1;
        for (int s = 0; s < nsteps; s++) {
          const char* cur = xl + (s & 1) * STAGE;
          char* nxt = xl + ((s + 1) & 1) * STAGE;
          const int kn = kb + (s + 2 < nsteps ? s + 2 : nsteps - 1) * X6BK;
          if constexpr (AMW == 0) {
#pragma unroll
            for (int c = 0; c < 4; c++) stage_part(c, nxt, kn);
          } else {
            bf16x8 bh[2], bm[2], bl[2];
            bf16x8 ah[2], am[2], al[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
              bh[j] = X6_FRAG(cur + 3 * PART + b_off[j]);
              bm[j] = X6_FRAG(cur + 4 * PART + b_off[j]);
              bl[j] = X6_FRAG(cur + 5 * PART + b_off[j]);
            }
            if constexpr (MODE == 2) {
#pragma unroll
              for (int p = 0; p < 4; p++) stage_part(p, nxt, kn);
            }
            ah[0] = X6_FRAG(cur + a_off[0]);
            am[0] = X6_FRAG(cur + PART + a_off[0]);
            al[0] = X6_FRAG(cur + 2 * PART + a_off[0]);
#pragma unroll
            for (int i = 0; i < AMW; i++) {
              if (i + 1 < AMW) {  // the next row's A fragments in flight under this row's MFMAs
                ah[(i + 1) & 1] = X6_FRAG(cur + a_off[i + 1]);
                am[(i + 1) & 1] = X6_FRAG(cur + PART + a_off[i + 1]);
                al[(i + 1) & 1] = X6_FRAG(cur + 2 * PART + a_off[i + 1]);
              }
              const int c = i & 1;
              if constexpr (STAGE_FIRST) {
#pragma unroll
                for (int p = i * 4 / AMW; p < (i + 1) * 4 / AMW; p++) stage_part(p, nxt, kn);
              }
#ifdef PCNN_X6_M16ABL  // timing ablation (wrong results): the same MFMA work as 16x16x32 instructions
#pragma unroll
              for (int j = 0; j < 2; j++) {
                const bf16x8 fa[6] = {al[c], ah[c], am[c], am[c], ah[c], ah[c]};
                const bf16x8 fb[6] = {bh[j], bl[j], bm[j], bh[j], bm[j], bh[j]};
#pragma unroll
                for (int p = 0; p < 12; p++)
                  a16[i][j][p & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[p >> 1], fb[p >> 1], a16[i][j][p & 3],
                                                                             0, 0, 0);
              }
              if (false)
#endif
#pragma unroll
              for (int j = 0; j < 2; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[c], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[c], bm[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[c], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], bm[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], bh[j], acc[i][j], 0, 0, 0);
              }
              if constexpr (MODE == 0) {
#pragma unroll
                for (int p = i * 4 / AMW; p < (i + 1) * 4 / AMW; p++) stage_part(p, nxt, kn);
              }
            }
            if constexpr (MODE == 3) {
#pragma unroll
              for (int p = 0; p < 4; p++) stage_part(p, nxt, kn);
            }
          }
          __syncthreads();
        }
      };
      // stagger: the two waves of a SIMD (wave w and w + 4: wm = 0 and 1) run
      // the same K step, so without an offset they reach their MFMAs and their
      // staging together (MI355X_MICROARCH.md, two waves per SIMD, item 9).
      // The wm = 1 waves stage first: all four parts before the rows where A
      // is k-contiguous (forward / dX shapes: half a step of offset), each
      // row's share before that row for the weight-gradient shapes, whose
      // row-contiguous operands take the longer offset badly.  Same-box A/B
      // (scripts/gemm_bench.py, nine GEMMs; the whole step 4007-4012 ->
      // 4156-4175 frames/s per-row, 4188-4198 half-step for every shape):
      // half-step fc6 fwd 494-503 -> 480-485, fc6 dX 471-473 -> 450, fc7 dX
      // 90 -> 82 us but fc6 dW 453 -> 477; per-row fc6 dW 453 -> 446 us.
      auto kloop_w = [&](auto amw_c) {
        if constexpr (A_T) {
          if (wm == 1) kloop(amw_c, IC<1>{});
          else kloop(amw_c, IC<0>{});
        } else {
          if (wm == 1) kloop(amw_c, IC<2>{});
          else kloop(amw_c, IC<3>{});
        }
      };
      if (amw == AM) kloop_w(IC<AM>{});
      else if (amw == 0) kloop_w(IC<0>{});
      else if (amw == 1) kloop_w(IC<1>{});
      else if constexpr (AM >= 4) {
        if (amw == 2) kloop_w(IC<2>{});
        else kloop_w(IC<3>{});
      }
    }
#ifdef PCNN_X6_M16ABL
#pragma unroll
    for (int i = 0; i < AM; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
          for (int e = 0; e < 4; e++) acc[i][j][4 * p + e] = a16[i][j][p][e];
#endif
    x_epilogue<T, AM>(g, pl, acc, m0, n0, rl, z, wm, wn, r, hsel);
  };

  const int kstep = (pl.ns + pl.S - 1) / pl.S;  // split-K: K steps per slice
  for (int item = wg; item < pl.tiles * pl.S; item += active) {
    const int z = item / pl.tiles, t = item % pl.tiles;
    const int kl = z * kstep;
    segment(t, kl, min(pl.ns, kl + kstep), z);
  }
}

template <int T, bool AT, bool BT, bool RG, bool S2, bool GN>
void launch_one(const GemmArgs& g, int grid, hipStream_t st) {
  // the attribute is per device: one flag per device ordinal
  static bool attr_set[pcnn::kMaxDevices] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= pcnn::kMaxDevices || !attr_set[dev]) {
    (void)hipFuncSetAttribute((const void*)k_gemm_x6<T, AT, BT, RG, S2, GN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, X6Tile<T>::lds);
    if (dev >= 0 && dev < pcnn::kMaxDevices) attr_set[dev] = true;
  }
  // the op's last launch when no reduce follows (gemm_impl holds the completion event back otherwise)
  pcnn::launch_last(k_gemm_x6<T, AT, BT, RG, S2, GN>, dim3(grid), dim3(X6Tile<T>::threads), X6Tile<T>::lds, st, g);
}

template <bool AT, bool BT, bool RG, bool S2>
void launch_tile(const GemmArgs& g, int grid, bool gen, hipStream_t st) {
  if (g.tile != 256) launch_one<128, AT, BT, RG, S2, true>(g, grid, st);
  else if (gen) launch_one<256, AT, BT, RG, S2, true>(g, grid, st);
  else launch_one<256, AT, BT, RG, S2, false>(g, grid, st);  // whole tiles only (static-M tile-mode shapes)
}

template <bool RG, bool S2>
void launch_layout(const GemmArgs& g, int grid, bool a_trans, bool b_trans, bool gen, hipStream_t st) {
  if (!a_trans && !b_trans) launch_tile<false, false, RG, S2>(g, grid, gen, st);
  else if (!a_trans && b_trans) launch_tile<false, true, RG, S2>(g, grid, gen, st);
  else if (a_trans && !b_trans) launch_tile<true, false, RG, S2>(g, grid, gen, st);
  else launch_tile<true, true, RG, S2>(g, grid, gen, st);
}

}  // namespace

namespace pcnn_gk {

void launch_gemm_x6(const GemmArgs& g, int grid, bool a_trans, bool b_trans, bool ragged, bool a2, bool gen,
                    hipStream_t st) {
  if (!ragged && !a2) launch_layout<false, false>(g, grid, a_trans, b_trans, gen, st);
  else if (!ragged) launch_layout<false, true>(g, grid, a_trans, b_trans, gen, st);
  else if (!a2) launch_layout<true, false>(g, grid, a_trans, b_trans, gen, st);
  else launch_layout<true, true>(g, grid, a_trans, b_trans, gen, st);
}

int gemm_x6_lds(int T) { return T == 256 ? X6Tile<256>::lds : X6Tile<128>::lds; }

}  // namespace pcnn_gk
