// The x6 GEMM on pre-split, fragment-tiled operand planes ("TP") staged by
// direct-to-LDS loads -- the fp32-faithful pose-head contraction with no
// split work inside the K loop.
//
// k_gemm_x6 (gemm_x6.hip) loads fp32 tiles into registers, splits every value
// into its bf16 hi / mid / lo planes and writes the six planes to LDS each K
// step: about a quarter of its time.  Here an operand arrives already split,
// in the layout the MFMA fragments read ("tiled planes"): for a matrix of
// `rows` x K (the M or N dimension x the contraction), block (rb, ks) of 32
// rows x 16 k is 3 KiB -- planes hi, mid, lo of 1 KiB each, and inside a plane
// lane l (0..63) owns 16 B: row 32 rb + (l & 31), k 16 ks + 8 (l >> 5) .. + 7
// as 8 bf16, exactly the v_mfma_f32_32x32x16_bf16 operand fragment of lane l.
// Blocks are stored row-block major, K steps contiguous:
//     offset(rb, ks, plane) = ((rb * ks_cap + ks) * 3 + plane) * 1 KiB.
// Rows past the matrix and k past the (device-side) contraction length hold
// zeros (the producer writes them), so partial tiles need no masks.
//
// One K step of a 256 x 256 tile is 48 such 1-KiB pieces (8 row blocks of A,
// 8 of B, 3 planes each); each of the 8 waves moves 6 with
// global_load_lds_dwordx4 (lane l's 16 B land at LDS base + 16 l: the piece
// IS the fragment image, so every ds_read_b128 is a linear, conflict-free
// 1 KiB read).  Three 48-KiB stages: the loads of step s + 2 are issued after
// the barrier of step s and stay in flight across it (counted vmcnt, raw
// s_barrier; cdna_hip_programming.md §5 "Pipelining across barriers"); the
// flat step sequence runs across tile boundaries, so the next tile's first
// two stages load during the current tile's last steps and its epilogue.
// The MFMA sequence per (row block, column block) and K step is k_gemm_x6's
// (lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi), and the plan, balanced M
// tiles, split-K slabs and epilogue are shared (gemm_common.h): results are
// bit-identical to k_gemm_x6 on the same fp32 operands.
#include "gemm_common.h"

using namespace pcnn_gk;

namespace {

constexpr int TT = 256;                     // tile edge
constexpr int kPiece = 1024;                // one plane of one (32 rows, 16 k) block
constexpr int kBlk3 = 3 * kPiece;
constexpr int kStage = 16 * kBlk3;          // 8 A + 8 B blocks, 48 KiB
constexpr int kNStage = 3;
constexpr int kLds = kNStage * kStage;      // 144 KiB
constexpr int kPiecesPerWave = 6;           // 48 pieces / 8 waves

struct TpArgs {
  GemmArgs g;
  const char* A;  // tiled planes of op(A): ceil(M / 32) row blocks x a_ks K steps
  const char* B;  // tiled planes of op(B)^T: ceil(N / 32) row blocks x b_ks K steps
  int a_ks, b_ks;
  int a_rb, b_rb;  // row blocks stored (loads past them are clamped; never read)
};

__device__ __forceinline__ void glds16(const char* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Where item it of this workgroup starts: (tile, slice, first step, steps)
struct Item {
  int t, z, kl, n;
};

#ifdef PCNN_TP_NOREAD  // timing ablation (wrong results): operands from registers, no LDS fragment reads
#define TP_FRAG(ptr) (fake)
#else
#define TP_FRAG(ptr) (*(const bf16x8*)(ptr))
#endif

template <bool GEN>
__global__ void __launch_bounds__(512, 1) k_gemm_tp(TpArgs p) {
  extern __shared__ __attribute__((aligned(16))) char xl[];
  const GemmArgs& g = p.g;
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  XPlan pl = x_plan(Meff, g.N, Keff, TT, g.xgrid, 16);
  if constexpr (!GEN) {
    pl.mode = 0;
    pl.S = 1;
  }
  const int total = pl.tiles * pl.S;
  const int active = min(g.xgrid, total);
  int wg = blockIdx.x;
  if (wg >= active) return;
  wg = xcd_remap(wg, active);
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  const int wm = wave / 4, wn = wave % 4;
  const int r = lane & 31, hsel = lane >> 5;
#ifdef PCNN_TP_NOREAD
  bf16x8 fake;
  for (int e = 0; e < 8; e++) fake[e] = (__bf16)(float)((lane * 7 + e) & 15);
#endif
  const int kstep = (pl.ns + pl.S - 1) / pl.S;
  auto item_of = [&](int it) {
    Item I;
    const int item = wg + it * active;
    I.z = item / pl.tiles;
    I.t = item % pl.tiles;
    I.kl = I.z * kstep;
    const int kh = min(pl.ns, I.kl + kstep);
    I.n = kh > I.kl ? kh - I.kl : 0;
    return I;
  };
  const int nitems = wg < total ? (total - 1 - wg) / active + 1 : 0;

  // the load cursor: (item, step within it), two flat steps ahead of compute
  int l_it = 0, l_s = 0;
  Item LI = item_of(0);
  // the cursor item's 6 source blocks of this wave (row-block base, K steps
  // stored), refreshed only when the cursor moves to another item
  const char* lsrc[kPiecesPerWave];
  auto set_item = [&]() {
    const int m0 = pl.mi_of(LI.t) * pl.Tm, n0 = pl.ni_of(LI.t) * TT;
#pragma unroll
    for (int u = 0; u < kPiecesPerWave; u++) {
      const int q = wave + 8 * u;  // piece 0..47: [A | B] x block x plane
      const int op = q / 24, rem = q % 24, blk = rem / 3, plane = rem % 3;
      if (op == 0) {
        const int rb = min(m0 / 32 + blk, p.a_rb - 1);
        lsrc[u] = p.A + ((size_t)(rb * p.a_ks + LI.kl) * 3 + plane) * kPiece + lane * 16;
      } else {
        const int rb = min(n0 / 32 + blk, p.b_rb - 1);
        lsrc[u] = p.B + ((size_t)(rb * p.b_ks + LI.kl) * 3 + plane) * kPiece + lane * 16;
      }
    }
  };
  auto skip_empty = [&]() {
    while (l_it < nitems && l_s >= LI.n) {
      l_it++;
      l_s = 0;
      if (l_it < nitems) {
        LI = item_of(l_it);
        set_item();
      }
    }
  };
  set_item();
  skip_empty();
  // issue this wave's 6 pieces of the cursor's step into stage `st`
  auto issue = [&](int st) {
    char* sb = xl + st * kStage;
#pragma unroll
    for (int u = 0; u < kPiecesPerWave; u++) {
      const int q = wave + 8 * u;
      const int op = q / 24, rem = q % 24, blk = rem / 3, plane = rem % 3;
      glds16(lsrc[u] + (size_t)l_s * kBlk3, sb + (op * 24 + blk * 3 + plane) * kPiece);
    }
    l_s++;
    skip_empty();
  };
  int issued = 0;  // flat steps issued
  if (l_it < nitems) { issue(0); issued++; }
  if (l_it < nitems) { issue(1); issued++; }

  int f = 0;  // flat step being computed
  for (int it = 0; it < nitems; it++) {
    const Item I = item_of(it);
    const int m0 = pl.mi_of(I.t) * pl.Tm, n0 = pl.ni_of(I.t) * TT;
    const int rl = min(Meff, m0 + pl.Tm);
    const int live = rl - (m0 + wm * (TT / 2));
    int amw = live <= 0 ? 0 : (live + 31) / 32;
    amw = __builtin_amdgcn_readfirstlane(amw < 4 ? amw : 4);
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = (f32x16){};
    auto kloop = [&](auto amw_c) {
      constexpr int AMW = decltype(amw_c)::value;
      for (int s = 0; s < I.n; s++, f++) {
        // this wave's pieces of step f landed (step f + 1's may still fly),
        // then every wave's, and every wave is done reading step f - 1's stage
#ifndef PCNN_TP_NOBAR
        if (issued > f + 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#endif
        if (l_it < nitems) {  // step f + 2 into the stage step f - 1 used
          issue((f + 2) % kNStage);
          issued++;
        }
        if constexpr (AMW > 0) {
          const char* cur = xl + (f % kNStage) * kStage;
          bf16x8 bh[2], bm[2], bl[2];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const char* bp = cur + (24 + (2 * wn + j) * 3) * kPiece + lane * 16;
            bh[j] = TP_FRAG(bp);
            bm[j] = TP_FRAG(bp + kPiece);
            bl[j] = TP_FRAG(bp + 2 * kPiece);
          }
#pragma unroll
          for (int i = 0; i < AMW; i++) {
            const char* ap = cur + ((4 * wm + i) * 3) * kPiece + lane * 16;
            const bf16x8 ah = TP_FRAG(ap);
            const bf16x8 am = TP_FRAG(ap + kPiece);
            const bf16x8 al = TP_FRAG(ap + 2 * kPiece);
#pragma unroll
            for (int j = 0; j < 2; j++) {  // smallest products first (k_gemm_x6's order)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
            }
          }
        }
      }
    };
    if (amw == 4) kloop(IC<4>{});
    else if (amw == 3) kloop(IC<3>{});
    else if (amw == 2) kloop(IC<2>{});
    else if (amw == 1) kloop(IC<1>{});
    else kloop(IC<0>{});
#ifdef PCNN_TP_NOEPI
    if (acc[0][0][0] == 1234.5f)  // ablation: stores only on an impossible value
#endif
    x_epilogue<TT, 4>(g, pl, acc, m0, n0, rl, I.z, wm, wn, r, hsel);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

// TP producer: one wave per (32-row block, 16-k step): lane l converts row
// 32 rb + (l & 31), k 16 ks + 8 (l >> 5) .. + 7 of the fp32 view
// src[row * rs + k * kst] (zeros past rows_eff / K_eff) into its 16 B of each
// plane.  Row blocks at or past ceil(rows_eff / 32) and K steps at or past
// ceil(K_eff / 16) are never multiplied and not written.
__global__ void __launch_bounds__(256) k_split_tp(const float* __restrict__ src, long rs, long kst, int rows,
                                                  const int32_t* __restrict__ rows_dev, int K,
                                                  const int32_t* __restrict__ K_dev, int n_rb, int ks_cap,
                                                  char* __restrict__ dst) {
  const int lane = pcnn::lane_id();
  const long chunk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (chunk >= (long)n_rb * ks_cap) return;
  const int rb = (int)(chunk / ks_cap), ks = (int)(chunk % ks_cap);
  const int Reff = eff_dim(rows, rows_dev), Keff = eff_dim(K, K_dev);
  // blocks wholly past the effective rows / K are never multiplied (the GEMM
  // skips dead row blocks and stops at ceil(K_eff / 16)): not written
  if ((ks * 16 >= Keff && ks > 0) || (rb * 32 >= Reff && rb > 0)) return;
  const int row = rb * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; e++) v[e] = (row < Reff && k0 + e < Keff) ? src[(size_t)row * rs + (size_t)(k0 + e) * kst] : 0.f;
  unsigned hi[4], mi[4], lo[4];
#pragma unroll
  for (int e = 0; e < 4; e++) x_split3(v[2 * e], v[2 * e + 1], hi[e], mi[e], lo[e]);
  char* o = dst + (size_t)chunk * kBlk3 + lane * 16;
  *(uint4*)(o) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
  *(uint4*)(o + kPiece) = make_uint4(mi[0], mi[1], mi[2], mi[3]);
  *(uint4*)(o + 2 * kPiece) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
}

template <bool GEN>
void launch_tp(const TpArgs& a, int grid, hipStream_t st) {
  static bool attr_set[pcnn::kMaxDevices] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= pcnn::kMaxDevices || !attr_set[dev]) {
    (void)hipFuncSetAttribute((const void*)k_gemm_tp<GEN>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (dev >= 0 && dev < pcnn::kMaxDevices) attr_set[dev] = true;
  }
  hipLaunchKernelGGL(k_gemm_tp<GEN>, dim3(grid), dim3(512), kLds, st, a);
}

}  // namespace

namespace pcnn_gk {
// k_gemm_reduce (pose_head.hip): split-K slabs + epilogue, dropout
void launch_gemm_reduce(const GemmArgs& g, hipStream_t st);
}

extern "C" size_t pcnn_tp_bytes(int rows, int K) {
  if (rows <= 0 || K <= 0) return 256;
  return (size_t)((rows + 31) / 32) * ((K + 15) / 16) * kBlk3;
}

extern "C" int pcnn_split_tp(const float* src, long row_stride, long k_stride, int rows, const int32_t* rows_dev, int K,
                             const int32_t* K_dev, void* dst, size_t dst_bytes, void* stream) {
  PCNN_REQUIRE(src && dst && rows > 0 && K > 0 && row_stride >= 0 && k_stride >= 0);
  PCNN_REQUIRE(dst_bytes >= pcnn_tp_bytes(rows, K) && ((uintptr_t)dst & 15) == 0);
  const int n_rb = (rows + 31) / 32, ks_cap = (K + 15) / 16;
  const long chunks = (long)n_rb * ks_cap;
  hipLaunchKernelGGL(k_split_tp, dim3((unsigned)((chunks + 3) / 4)), dim3(256), 0, (hipStream_t)stream, src,
                     row_stride, k_stride, rows, rows_dev, K, K_dev, n_rb, ks_cap, (char*)dst);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_gemm_tp(int M, int N, int K, const void* A_tp, const void* B_tp, float* Cm, int ldc,
                            const float* bias, int act, const float* mask, int ldm, const uint8_t* drop, int ldd,
                            float keep_prob, const int32_t* M_dev, const int32_t* K_dev, void* workspace,
                            size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(M >= 0 && N > 0 && K > 0 && A_tp && B_tp && Cm && ldc >= N && (act == 0 || act == 1));
  PCNN_REQUIRE(!mask || ldm >= N);
  PCNN_REQUIRE(keep_prob > 0.f && keep_prob <= 1.f && (!drop || ldd >= N));
  PCNN_REQUIRE(((uintptr_t)A_tp & 15) == 0 && ((uintptr_t)B_tp & 15) == 0);
  PCNN_REQUIRE((long)M * ldc < (1l << 29) && (!mask || (long)M * ldm < (1l << 29)));
  if (M == 0) return PCNN_OK;
  if (workspace_bytes < pcnn_gemm_workspace_size(M, N, K, M_dev != nullptr, 2) || !workspace) return PCNN_ECAPACITY;
  GemmArgs g{M, N, K, nullptr, nullptr, 0, nullptr, 0, Cm, ldc, bias, act, mask, ldm, M_dev, K_dev,
             (float*)workspace, 2, TT, 0, 0, drop, ldd, keep_prob};
  const int max_grid = 256;
  long grid = max_grid;
  bool gen = true, may_split = true;
  if (!M_dev) {  // as pcnn_gemm: static M -> fewest workgroups that keep the rounds
    const XPlan pl = x_plan(M, N, K, TT, max_grid, 16);
    may_split = pl.mode == 1;
    if (pl.mode == 0) {
      gen = false;
      const long items = pl.tiles;
      const long rounds = (items + max_grid - 1) / max_grid;
      grid = (items + rounds - 1) / rounds;
      grid = (grid + 7) / 8 * 8;
      if (grid > max_grid) grid = max_grid;
    }
  }
  g.xgrid = (int)grid;
  g.c_stream = (long)M * N * 4 > (256l << 20);
  TpArgs a{g, (const char*)A_tp, (const char*)B_tp, (K + 15) / 16, (K + 15) / 16, (M + 31) / 32, (N + 31) / 32};
  hipStream_t st = (hipStream_t)stream;
  if (gen) launch_tp<true>(a, (int)grid, st);
  else launch_tp<false>(a, (int)grid, st);
  if (may_split || drop || keep_prob != 1.f) launch_gemm_reduce(g, st);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
