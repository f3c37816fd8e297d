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
#include "pcnn_common.h"
#include <math.h>

namespace {

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int kGemmThreads = 256;
constexpr int kMaxSplit = 8;

typedef float f32x16 __attribute__((ext_vector_type(16)));

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
  float* slab;  // split-K partials [kMaxSplit][M][N]
};

__device__ __forceinline__ int eff_dim(int full, const int32_t* dev) {
  if (!dev) return full;
  int v = *dev;
  return v < full ? (v < 0 ? 0 : v) : full;
}

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

__global__ void __launch_bounds__(256) k_gemm_reduce(GemmArgs g) {
  const int Meff = eff_dim(g.M, g.M_dev);
  const int Keff = eff_dim(g.K, g.K_dev);
  const int S = split_for(Meff, g.N, Keff);
  if (S == 1) return;
  const long total = (long)Meff * g.N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / g.N), n = (int)(i % g.N);
    float v = 0.f;
    for (int z = 0; z < S; z++) v += g.slab[((size_t)z * g.M + m) * g.N + n];
    g.C[(size_t)m * g.ldc + n] = epilogue(v, g, m, n);
  }
}

__global__ void k_colsum(const float* __restrict__ X, int M, int N, int ldx, const int32_t* __restrict__ M_dev,
                         float* __restrict__ out) {
  const int Meff = eff_dim(M, M_dev);
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int m = 0; m < Meff; m++) s += X[(size_t)m * ldx + n];
    out[n] = s;
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
                                                   float* __restrict__ dy8) {
  const int R = eff_dim(R_cap, num_rois_dev);
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = pcnn::lane_id();
  if (row >= R) return;
  float ss = 0.f, dot = 0.f;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    if (c < D) {
      const float mv = t_in[(size_t)row * D + c] * pw[(size_t)row * D + c];
      ss += mv * mv;
      dot += pred[(size_t)row * D + c] * dpred[(size_t)row * D + c];
    }
  }
  ss = pcnn::wave_sum(ss);
  dot = pcnn::wave_sum(dot);
  const bool clamp = !(ss > 1e-12f);
  const float inv = 1.f / sqrtf(fmaxf(ss, 1e-12f));
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = lane + 64 * k;
    if (c < D) {
      const size_t o = (size_t)row * D + c;
      // d/dm of m * rsqrt(max(sum m^2, eps))
      const float dm = clamp ? dpred[o] * inv : (dpred[o] - pred[o] * dot) * inv;
      const float dt = dm * pw[o];
      const float t = t_in[o];
      dy8[o] = dt * (1.f - t * t);
    }
  }
}

}  // namespace

extern "C" size_t pcnn_gemm_workspace_size(int M, int N, int K, int m_dynamic, int precision) {
  (void)precision;
  if (M <= 0 || N <= 0) return 256;
  // split-K partial slabs; the split only grows when the device-side M shrinks
  const int s = split_for(m_dynamic ? 1 : M, N, K);
  return s > 1 ? pcnn::align_up((size_t)s * M * N * sizeof(float), 256) + 256 : 256;
}

extern "C" int pcnn_gemm(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B,
                         int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act, const float* mask,
                         int ldm, const int32_t* M_dev, const int32_t* K_dev, int precision, void* workspace,
                         size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(M >= 0 && N > 0 && K >= 0 && A && B && Cm);
  PCNN_REQUIRE(precision == 0);
  PCNN_REQUIRE(lda >= (a_trans ? M : K) && ldb >= (b_trans ? K : N) && ldc >= N);
  PCNN_REQUIRE(!mask || ldm >= N);
  PCNN_REQUIRE(act == 0 || act == 1);
  if (M == 0) return PCNN_OK;
  if (workspace_bytes < pcnn_gemm_workspace_size(M, N, K, M_dev != nullptr, precision) || !workspace)
    return PCNN_ECAPACITY;
  GemmArgs g{M, N, K, A, A2, lda, B, ldb, Cm, ldc, bias, act, mask, ldm, M_dev, K_dev, (float*)workspace};
  hipStream_t st = (hipStream_t)stream;
  const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  // persistent grid sized for the capacity shape at its split
  const long items = (long)mt * nt * split_for(M, N, K);
  long grid = items < 2048 ? items : 2048;
  if (grid < 512) grid = 512;
  if (!a_trans && !b_trans) hipLaunchKernelGGL((k_gemm_f32<false, false>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else if (!a_trans && b_trans) hipLaunchKernelGGL((k_gemm_f32<false, true>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else if (a_trans && !b_trans) hipLaunchKernelGGL((k_gemm_f32<true, false>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  else hipLaunchKernelGGL((k_gemm_f32<true, true>), dim3(grid), dim3(kGemmThreads), 0, st, g);
  hipLaunchKernelGGL(k_gemm_reduce, dim3(1024), dim3(256), 0, st, g);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_colsum(const float* X, int M, int N, int ldx, const int32_t* M_dev, float* out, void* stream) {
  PCNN_REQUIRE(X && out && M >= 0 && N > 0 && ldx >= N);
  hipLaunchKernelGGL(k_colsum, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, X, M, N, ldx, M_dev, out);
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

extern "C" int pcnn_pose_head_bwd(const float* d_pred, const float* tanh_out, const float* poses_weight,
                                  const float* pred, int R_cap, const int32_t* num_rois_dev, int D, float* d_y8,
                                  void* stream) {
  PCNN_REQUIRE(d_pred && tanh_out && poses_weight && pred && d_y8 && R_cap >= 0 && D > 0 && D <= 256);
  if (R_cap == 0) return PCNN_OK;
  hipLaunchKernelGGL(k_head_bwd, dim3((R_cap + 3) / 4), dim3(256), 0, (hipStream_t)stream, d_pred, tanh_out,
                     poses_weight, pred, R_cap, num_rois_dev, D, d_y8);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
