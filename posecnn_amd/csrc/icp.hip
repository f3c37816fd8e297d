// Test-time pose refinement on MI355X: the numerical
// core of Synthesizer::solveICP (lib/synthesize/synthesize.cpp:2052-2395),
// called from lib/fcn/test.py:1316-1351 through synthesizer.icp_python.
//
//   pcnn_icp_live_vertices   masked depth -> live vertex map per object
//                            (synthesize.cpp:2140-2160 + df::backproject,
//                            lib/kinect_fusion/src/image/backprojection.cu:10-27)
//   pcnn_icp_center          translation re-centring (synthesize.cpp:2163-2233)
//   pcnn_pose_energy         optEnergy of K candidate poses (synthesize.cpp:2474-2526)
//   pcnn_icp                 df::icp (lib/kinect_fusion/src/optimization/icp.cpp:20-106,
//                            icp.cu:22-245), batched over N (RoI, hypothesis) problems
//
// The reference runs each ICP iteration as a per-pixel kernel over the whole
// H x W frame that writes a Jacobian row per pixel to HBM, a thrust
// transform_reduce of those rows, a device sync and a host-side 6x6 LDLT solve
// (icp.cpp:51-103).  Here the pixels whose rendered depth lies in the depth
// range (the only ones icpKernel can use: icp.cu:56-63) are compacted once per
// problem, in raster order, into dense (vertex, normal) records; then each
// Gauss-Newton iteration is one launch over all N problems: 8-64 workgroups
// per problem each first finish the previous iteration (its slices added in
// order, the 6x6 system solved by Eigen's LDLT with diagonal pivoting, the
// twist exponentiated by Sophus SE3::exp and left-multiplied into the
// accumulated update -- redundantly and identically in every workgroup), then
// accumulate J^T J and J^T r in registers and reduce them through the wave and
// the workgroup into their slice of the iteration's system.  No per-pixel Jacobian ever
// reaches HBM and the host is never involved.
//
// Rendering (the OpenGL vertex / normal / canonical-coordinate maps of the
// model at a pose, synthesize.cpp:2106-2137) and the NLopt Nelder-Mead pose
// search (poseWithOpt, :2529-2573) are outside the path: the maps are inputs.
#include "pcnn_common.h"

namespace pcnn_refine {

constexpr int kSeg = 2048;       // pixels per compaction / reduction block
constexpr int kBlk = 256;        // threads of the per-pixel kernels
constexpr int kSys = 28;         // 21 upper-triangle JTJ + 6 JTr + pixel count

struct Quat { float w, x, y, z; };
struct SE3 { Quat q; float t[3]; };

// Eigen Quaternion::_transformVector (the point action of Sophus SO3)
__device__ __forceinline__ void rotate(const Quat& q, float v0, float v1, float v2, float& o0, float& o1,
                                       float& o2) {
  float uv0 = q.y * v2 - q.z * v1;
  float uv1 = q.z * v0 - q.x * v2;
  float uv2 = q.x * v1 - q.y * v0;
  uv0 = uv0 + uv0;
  uv1 = uv1 + uv1;
  uv2 = uv2 + uv2;
  const float c0 = q.y * uv2 - q.z * uv1;
  const float c1 = q.z * uv0 - q.x * uv2;
  const float c2 = q.x * uv1 - q.y * uv0;
  o0 = v0 + q.w * uv0 + c0;
  o1 = v1 + q.w * uv1 + c1;
  o2 = v2 + q.w * uv2 + c2;
}

// Sophus SE3 product a * b (quaternion renormalised by 2 / (1 + |q|^2))
__device__ SE3 se3_mul(const SE3& a, const SE3& b) {
  SE3 r;
  float t0, t1, t2;
  rotate(a.q, b.t[0], b.t[1], b.t[2], t0, t1, t2);
  r.t[0] = a.t[0] + t0;
  r.t[1] = a.t[1] + t1;
  r.t[2] = a.t[2] + t2;
  r.q.w = a.q.w * b.q.w - a.q.x * b.q.x - a.q.y * b.q.y - a.q.z * b.q.z;
  r.q.x = a.q.w * b.q.x + a.q.x * b.q.w + a.q.y * b.q.z - a.q.z * b.q.y;
  r.q.y = a.q.w * b.q.y + a.q.y * b.q.w + a.q.z * b.q.x - a.q.x * b.q.z;
  r.q.z = a.q.w * b.q.z + a.q.z * b.q.w + a.q.x * b.q.y - a.q.y * b.q.x;
  const float n2 = r.q.w * r.q.w + r.q.x * r.q.x + r.q.y * r.q.y + r.q.z * r.q.z;
  if (n2 != 1.0f) {
    const float s = 2.0f / (1.0f + n2);
    r.q.w *= s;
    r.q.x *= s;
    r.q.y *= s;
    r.q.z *= s;
  }
  return r;
}

// Sophus SE3<float>::exp of the twist (upsilon, omega)
__device__ SE3 se3_exp(const float a[6]) {
  const float w0 = a[3], w1 = a[4], w2 = a[5];
  const float theta_sq = w0 * w0 + w1 * w1 + w2 * w2;
  const float theta = sqrtf(theta_sq);
  const float eps = 1e-5f;
  float imag, real;
  if (theta < eps) {
    const float t4 = theta_sq * theta_sq;
    imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * t4;
    real = 1.0f - 0.5f * theta_sq + (float)(1.0 / 384.0) * t4;
  } else {
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  SE3 r;
  r.q = {real, imag * w0, imag * w1, imag * w2};
  float V[9];
  if (theta < eps) {  // V = so3.matrix()
    const Quat& q = r.q;
    const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z;
    const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    V[0] = 1.f - (tyy + tzz); V[1] = txy - twz; V[2] = txz + twy;
    V[3] = txy + twz; V[4] = 1.f - (txx + tzz); V[5] = tyz - twx;
    V[6] = txz - twy; V[7] = tyz + twx; V[8] = 1.f - (txx + tyy);
  } else {
    const float O[9] = {0.f, -w2, w1, w2, 0.f, -w0, -w1, w0, 0.f};
    const float c1 = (1.0f - cosf(theta)) / theta_sq;
    const float c2 = (theta - sinf(theta)) / (theta_sq * theta);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const float o2 = O[i * 3 + 0] * O[0 * 3 + j] + O[i * 3 + 1] * O[1 * 3 + j] + O[i * 3 + 2] * O[2 * 3 + j];
        V[i * 3 + j] = (i == j ? 1.f : 0.f) + c1 * O[i * 3 + j] + c2 * o2;
      }
  }
#pragma unroll
  for (int i = 0; i < 3; i++) r.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
  return r;
}

// Eigen 3.3 LDLT<Upper> of the symmetric 6x6 system and its solve
// (diagonal pivoting; zero pivots -> 0 in the pseudo-inverse of D).  Every
// loop is unrolled so that each matrix index is a compile-time constant and m
// stays in registers; the data-dependent pivot swaps become selects over the
// candidate rows.
template <int K, int BI>
__device__ __forceinline__ void ldlt_swap(float (&m)[36]) {
#pragma unroll
  for (int j = 0; j < K; j++) { const float t = m[K * 6 + j]; m[K * 6 + j] = m[BI * 6 + j]; m[BI * 6 + j] = t; }
#pragma unroll
  for (int i = BI + 1; i < 6; i++) { const float t = m[i * 6 + K]; m[i * 6 + K] = m[i * 6 + BI]; m[i * 6 + BI] = t; }
  { const float t = m[K * 6 + K]; m[K * 6 + K] = m[BI * 6 + BI]; m[BI * 6 + BI] = t; }
#pragma unroll
  for (int i = K + 1; i < BI; i++) { const float t = m[i * 6 + K]; m[i * 6 + K] = m[BI * 6 + i]; m[BI * 6 + i] = t; }
}

template <int K>
__device__ __forceinline__ void ldlt_pivot(float (&m)[36], int big) {
  if constexpr (K + 1 < 6) { if (big == K + 1) ldlt_swap<K, K + 1>(m); }
  if constexpr (K + 2 < 6) { if (big == K + 2) ldlt_swap<K, K + 2>(m); }
  if constexpr (K + 3 < 6) { if (big == K + 3) ldlt_swap<K, K + 3>(m); }
  if constexpr (K + 4 < 6) { if (big == K + 4) ldlt_swap<K, K + 4>(m); }
  if constexpr (K + 5 < 6) { if (big == K + 5) ldlt_swap<K, K + 5>(m); }
}

// x[k] <-> x[t] for a runtime t >= k
template <int K>
__device__ __forceinline__ void swap_x(float (&x)[6], int t) {
#pragma unroll
  for (int i = K + 1; i < 6; i++)
    if (t == i) { const float v = x[K]; x[K] = x[i]; x[i] = v; }
}

template <int K>
__device__ __forceinline__ bool ldlt_step(float (&m)[36], int (&tr)[6]) {
  int big = K;
  float bv = fabsf(m[K * 6 + K]);
#pragma unroll
  for (int i = K + 1; i < 6; i++)
    if (fabsf(m[i * 6 + i]) > bv) {
      bv = fabsf(m[i * 6 + i]);
      big = i;
    }
  tr[K] = big;
  ldlt_pivot<K>(m, big);
  if constexpr (K > 0) {
    float temp[K > 0 ? K : 1];
#pragma unroll
    for (int j = 0; j < K; j++) temp[j] = m[j * 6 + j] * m[K * 6 + j];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < K; j++) sum = sum + m[K * 6 + j] * temp[j];
    m[K * 6 + K] -= sum;
#pragma unroll
    for (int i = K + 1; i < 6; i++) {
      float si = 0.f;
#pragma unroll
      for (int j = 0; j < K; j++) si = si + m[i * 6 + j] * temp[j];
      m[i * 6 + K] -= si;
    }
  }
  const float akk = m[K * 6 + K];
  const bool valid = fabsf(akk) > 0.f;
  if (K == 0 && !valid) return false;  // all-zero diagonal: nothing to solve
  if (K < 5 && valid) {
#pragma unroll
    for (int i = K + 1; i < 6; i++) m[i * 6 + K] /= akk;
  }
  return true;
}

__device__ void ldlt_solve6(float (&m)[36], const float (&b)[6], float (&x)[6]) {
  int tr[6];
  if (!ldlt_step<0>(m, tr)) {
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = 0.f;
    return;
  }
  ldlt_step<1>(m, tr);
  ldlt_step<2>(m, tr);
  ldlt_step<3>(m, tr);
  ldlt_step<4>(m, tr);
  ldlt_step<5>(m, tr);
#pragma unroll
  for (int i = 0; i < 6; i++) x[i] = b[i];
  swap_x<0>(x, tr[0]); swap_x<1>(x, tr[1]); swap_x<2>(x, tr[2]);
  swap_x<3>(x, tr[3]); swap_x<4>(x, tr[4]); swap_x<5>(x, tr[5]);
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < i; j++) x[i] -= m[i * 6 + j] * x[j];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const float d = m[i * 6 + i];
    x[i] = fabsf(d) > 1.17549435e-38f ? x[i] / d : 0.f;
  }
#pragma unroll
  for (int i = 5; i >= 0; i--)
#pragma unroll
    for (int j = i + 1; j < 6; j++) x[i] -= m[j * 6 + i] * x[j];
  swap_x<5>(x, tr[5]); swap_x<4>(x, tr[4]); swap_x<3>(x, tr[3]);
  swap_x<2>(x, tr[2]); swap_x<1>(x, tr[1]); swap_x<0>(x, tr[0]);
}


// sum of n strided floats in index order, loads issued 8 ahead of the adds
// (a plain loop waits out one memory latency per term)
__device__ __forceinline__ float ordered_sum_strided(const float* __restrict__ p, int n, size_t stride) {
  float sum = 0.f;
  for (int q0 = 0; q0 < n; q0 += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = q0 + k < n ? p[(size_t)(q0 + k) * stride] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (q0 + k < n) sum += v[k];
  }
  return sum;
}

__device__ __forceinline__ bool in_range(float z, float znear, float zfar) { return !(z < znear || z > zfar); }

// Block-wide sum of an int (all threads call; result in every thread).
template <int T>
__device__ __forceinline__ int block_sum_int(int v, int* sh) {
  v = pcnn::wave_sum(v);
  if (pcnn::lane_id() == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int w = 0; w < T / 64; w++) s += sh[w];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// live vertices: one thread per 4 pixels of one object's map (float4 stores)
__global__ void __launch_bounds__(kBlk) k_icp_live(const uint16_t* __restrict__ depth,
                                                   const int32_t* __restrict__ label, int HW, int W,
                                                   const int32_t* __restrict__ obj_ids, float factor, float fx,
                                                   float fy, float px, float py, float* __restrict__ out) {
  const int l = blockIdx.y;
  const int obj = obj_ids[l];
  const int p0 = 4 * (blockIdx.x * kBlk + threadIdx.x);
  if (p0 >= HW) return;
  float v[12];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int p = p0 + e;
    float d = 0.f;
    int x = 0, y = 0;
    if (p < HW) {
      d = label[p] == obj ? (float)depth[p] / factor : 0.f;
      x = p % W;
      y = p / W;
    }
    v[3 * e + 0] = (((float)x - px) / fx) * d;
    v[3 * e + 1] = (((float)y - py) / fy) * d;
    v[3 * e + 2] = d;
  }
  float* o = out + ((size_t)l * HW + p0) * 3;
  if (p0 + 4 <= HW) {
    float4* o4 = (float4*)o;  // HW % 4 == 0 is required by the launcher
    o4[0] = make_float4(v[0], v[1], v[2], v[3]);
    o4[1] = make_float4(v[4], v[5], v[6], v[7]);
    o4[2] = make_float4(v[8], v[9], v[10], v[11]);
  }
}

// compaction pass 1: per (segment, problem) the count of pixels whose rendered
// depth is in range
__global__ void __launch_bounds__(kBlk) k_icp_count(const float* __restrict__ pred_v, int HW, float znear,
                                                    float zfar, int nseg, int32_t* __restrict__ cnt) {
  __shared__ int sh[kBlk / 64];
  const int n = blockIdx.y, seg = blockIdx.x;
  const float* pv = pred_v + (size_t)n * HW * 4;
  int c = 0;
  for (int i = threadIdx.x; i < kSeg; i += kBlk) {
    const int p = seg * kSeg + i;
    if (p < HW && in_range(pv[(size_t)p * 4 + 2], znear, zfar)) c++;
  }
  c = block_sum_int<kBlk>(c, sh);
  if (threadIdx.x == 0) cnt[(size_t)n * nseg + seg] = c;
}

// compaction pass 2: the segment's in-range pixels in raster order ->
// records [offset, offset + count) of problem n (rec[2i] = vertex, rec[2i+1] =
// normal)
__global__ void __launch_bounds__(kBlk) k_icp_scatter(const float* __restrict__ pred_v,
                                                      const float* __restrict__ pred_n, int HW, float znear,
                                                      float zfar, int nseg, const int32_t* __restrict__ cnt,
                                                      float4* __restrict__ rec) {
  __shared__ int sh[kBlk / 64];
  __shared__ int wc[kBlk / 64];
  const int n = blockIdx.y, seg = blockIdx.x;
  const int32_t* cn = cnt + (size_t)n * nseg;
  int o = 0;
  for (int s = threadIdx.x; s < seg; s += kBlk) o += cn[s];
  int off = block_sum_int<kBlk>(o, sh);
  const float4* pv = (const float4*)(pred_v + (size_t)n * HW * 4);
  const float4* pn = (const float4*)(pred_n + (size_t)n * HW * 4);
  float4* rn = rec + (size_t)n * HW * 2;
  const int wave = threadIdx.x >> 6;
  for (int i0 = 0; i0 < kSeg; i0 += kBlk) {
    const int p = seg * kSeg + i0 + threadIdx.x;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    bool ok = false;
    if (p < HW) {
      v = pv[p];
      ok = in_range(v.z, znear, zfar);
    }
    const uint64_t m = __ballot(ok);
    if (pcnn::lane_id() == 0) wc[wave] = __popcll(m);
    __syncthreads();
    int base = off;
    for (int w = 0; w < wave; w++) base += wc[w];
    if (ok) {
      const int r = base + __popcll(m & pcnn::lanemask_lt());
      rn[2 * (size_t)r] = v;
      rn[2 * (size_t)r + 1] = pn[p];
    }
    for (int w = 0; w < kBlk / 64; w++) off += wc[w];
    __syncthreads();
  }
}


// T_next = exp(LDLT solve of the 28-entry system) * T  (one lane)
__device__ SE3 icp_advance(const float* sys, const SE3& T) {
  float m[36], b[6], x[6];
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = i; j < 6; j++) {
      m[i * 6 + j] = sys[k];
      m[j * 6 + i] = sys[k];
      k++;
    }
#pragma unroll
  for (int i = 0; i < 6; i++) b[i] = sys[21 + i];
  ldlt_solve6(m, b, x);
  return se3_mul(se3_exp(x), T);
}

// One Gauss-Newton iteration of df::icp for N problems: grid (split, N).
// Each workgroup first finishes the previous iteration itself -- the slices
// of its system added in slice order, the LDLT solve and exp(x) applied to
// the previous pose, identically in every workgroup (workgroup 0 publishes
// the pose for the next launch) -- then accumulates J^T J / J^T r over a
// strided slice of its problem's records into its slot of this iteration's
// `partial` buffer (double-buffered); k_icp_finish solves the last one.  The
// order of every sum is fixed (lane, wave tree, waves, slices): results are
// run-to-run identical.  (Measured alternatives: a last-arriver ticket that
// solves inside the iteration, 28 us per iteration at 16 slices and 65 at 64
// -- each workgroup's device-scope release fence costs more than a launch;
// a separate one-wave solve launch per iteration, 185 vs 163 us per 8 x 8.)
constexpr int kIcpSplitMax = 64;  // workgroups per problem (the launcher picks 8..64 by N)

__device__ __forceinline__ SE3 load_se3(const float* p) {
  SE3 T;
  T.q = {p[0], p[1], p[2], p[3]};
  T.t[0] = p[4]; T.t[1] = p[5]; T.t[2] = p[6];
  return T;
}
__device__ __forceinline__ void store_se3(float* p, const SE3& T) {
  p[0] = T.q.w; p[1] = T.q.x; p[2] = T.q.y; p[3] = T.q.z;
  p[4] = T.t[0]; p[5] = T.t[1]; p[6] = T.t[2];
}

__global__ void __launch_bounds__(kBlk) k_icp_step(
    const float4* __restrict__ rec, const int32_t* __restrict__ cnt, int nseg, const float* __restrict__ live,
    const int32_t* __restrict__ live_index, int num_live, int H, int W, float fx, float fy, float px, float py,
    float znear, float zfar, float max_error, int it, int iterations, int split, float* __restrict__ acc_pose,
    float* __restrict__ partial, float* __restrict__ systems) {
  __shared__ float part[kBlk / 64][kSys];
  __shared__ int ish[kBlk / 64];
  __shared__ float psys[kSys];
  __shared__ SE3 Tsh;
  const int n = blockIdx.y, g = blockIdx.x;
  const int HW = H * W;
  const size_t pstride = (size_t)kIcpSplitMax * kSys;  // one problem's slices
  int c = 0;
  for (int s = threadIdx.x; s < nseg; s += kBlk) c += cnt[(size_t)n * nseg + s];
  const int li = live_index ? live_index[n] : n;
  // a live index outside [0, num_live) contributes no pixel (identity update)
  const int total = (li >= 0 && li < num_live) ? block_sum_int<kBlk>(c, ish) : (block_sum_int<kBlk>(0, ish), 0);
  const float4* rn = rec + (size_t)n * HW * 2;
  const float* lv = live + (size_t)(li >= 0 && li < num_live ? li : 0) * HW * 3;
  if (it > 0) {  // finish iteration it - 1
    const float* pp = partial + ((size_t)((it - 1) & 1) * gridDim.y + n) * pstride;
    if (threadIdx.x < kSys) psys[threadIdx.x] = ordered_sum_strided(pp + threadIdx.x, split, kSys);
    __syncthreads();
    if (threadIdx.x == 0) {
      const SE3 Tp = it == 1 ? SE3{{1.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}
                             : load_se3(acc_pose + ((size_t)((it - 1) & 1) * gridDim.y + n) * 8);
      Tsh = icp_advance(psys, Tp);
      if (g == 0) store_se3(acc_pose + ((size_t)(it & 1) * gridDim.y + n) * 8, Tsh);
    }
    if (g == 0 && systems && threadIdx.x < kSys)
      systems[((size_t)n * iterations + it - 1) * kSys + threadIdx.x] = psys[threadIdx.x];
  } else if (threadIdx.x == 0) {
    Tsh = SE3{{1.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
  }
  __syncthreads();
  const SE3 T = Tsh;
  const float border = 2.f;
  const float umax = (float)(W - 1) - border, vmax = (float)(H - 1) - border;
  const int wave = threadIdx.x >> 6, lane = pcnn::lane_id();
  float a[kSys];
#pragma unroll
  for (int e = 0; e < kSys; e++) a[e] = 0.f;
  const int stride = split * kBlk;
  int i = g * kBlk + threadIdx.x;
  float4 vn = make_float4(0.f, 0.f, 0.f, 0.f), nn = vn;
  if (i < total) {
    vn = rn[2 * (size_t)i];
    nn = rn[2 * (size_t)i + 1];
  }
  for (; i < total; i += stride) {
    const float4 v = vn, nm = nn;  // the next record is in flight under this one's work
    if (i + stride < total) {
      vn = rn[2 * ((size_t)i + stride)];
      nn = rn[2 * ((size_t)i + stride) + 1];
    }
    float p0, p1, p2;
    rotate(T.q, v.x, v.y, v.z, p0, p1, p2);
    p0 = p0 + T.t[0];
    p1 = p1 + T.t[1];
    p2 = p2 + T.t[2];
    const int u = (int)((p0 / p2) * fx + px + 0.5f);  // v_cvt_i32_f32: NaN -> 0
    const int vv = (int)((p1 / p2) * fy + py + 0.5f);
    if ((float)u <= border || (float)u >= umax || (float)vv <= border || (float)vv >= vmax) continue;
    const float* l3 = lv + ((size_t)vv * W + u) * 3;
    const float l0 = l3[0], l1 = l3[1], l2 = l3[2];
    if (l2 < znear || l2 > zfar) continue;
    const float nr = sqrtf(p0 * p0 + p1 * p1 + p2 * p2);
    if (-((p0 / nr) * nm.x + (p1 / nr) * nm.y + (p2 / nr) * nm.z) < 0.1f) continue;
    const float e = nm.x * (l0 - p0) + nm.y * (l1 - p1) + nm.z * (l2 - p2);
    if (fabsf(e) > max_error) continue;
    const float w = 1.0f / l2;
    float J[6];
    J[0] = w * nm.x;
    J[1] = w * nm.y;
    J[2] = w * nm.z;
    J[3] = w * (nm.z * p1 - nm.y * p2);
    J[4] = w * (nm.x * p2 - nm.z * p0);
    J[5] = w * (nm.y * p0 - nm.x * p1);
    const float r = w * e;
    int k = 0;
#pragma unroll
    for (int ii = 0; ii < 6; ii++)
#pragma unroll
      for (int jj = ii; jj < 6; jj++) a[k++] += J[ii] * J[jj];
#pragma unroll
    for (int ii = 0; ii < 6; ii++) a[21 + ii] += J[ii] * r;
    a[27] += 1.f;
  }
#pragma unroll
  for (int e = 0; e < kSys; e++) {
    const float sum = pcnn::wave_sum(a[e]);
    if (lane == 0) part[wave][e] = sum;
  }
  __syncthreads();
  if (threadIdx.x < kSys) {
    float sum = 0.f;
    for (int w = 0; w < kBlk / 64; w++) sum += part[w][threadIdx.x];
    partial[((size_t)(it & 1) * gridDim.y + n) * pstride + (size_t)g * kSys + threadIdx.x] = sum;
  }
}

// The last iteration's solve, one wave per problem: its slices added in
// order, the update and (optionally) update * pose_in written out.
__global__ void __launch_bounds__(64) k_icp_finish(int N, int iterations, int split, const float* __restrict__ acc_pose,
                                                   const float* __restrict__ partial, const float* __restrict__ pose_in,
                                                   float* __restrict__ update, float* __restrict__ pose_out,
                                                   float* __restrict__ systems) {
  __shared__ float sys[kSys];
  const int n = blockIdx.x, it = iterations - 1;
  const float* pp = partial + ((size_t)(it & 1) * N + n) * (size_t)kIcpSplitMax * kSys;
  if (threadIdx.x < kSys) {
    sys[threadIdx.x] = ordered_sum_strided(pp + threadIdx.x, split, kSys);
    if (systems) systems[((size_t)n * iterations + it) * kSys + threadIdx.x] = sys[threadIdx.x];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const SE3 Tp = it == 0 ? SE3{{1.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}} : load_se3(acc_pose + ((size_t)(it & 1) * N + n) * 8);
  const SE3 A = icp_advance(sys, Tp);
  store_se3(update + (size_t)n * 7, A);
  if (pose_in && pose_out) {  // refinePose: T_co = update * T_co (synthesize.cpp:2023-2025)
    const float* P = pose_in + (size_t)n * 7;
    const float qn = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
    SE3 B;
    B.q = {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
    B.t[0] = P[4]; B.t[1] = P[5]; B.t[2] = P[6];
    store_se3(pose_out + (size_t)n * 7, se3_mul(A, B));
  }
}

// iterations == 0: the identity update (and pose_out = pose_in, normalised)
__global__ void k_icp_identity(int N, const float* __restrict__ pose_in, float* __restrict__ update,
                               float* __restrict__ pose_out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  store_se3(update + (size_t)n * 7, SE3{{1.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}});
  if (pose_in && pose_out) {
    const float* P = pose_in + (size_t)n * 7;
    const float qn = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
    float* o = pose_out + (size_t)n * 7;
    o[0] = P[0] / qn; o[1] = P[1] / qn; o[2] = P[2] / qn; o[3] = P[3] / qn;
    o[4] = P[4]; o[5] = P[5]; o[6] = P[6];
  }
}

// ---------------------------------------------------------------------------
// Segmented sums with a fixed-order finish: every block writes its partial,
// the last block to arrive (ticket) adds the partials in block order.
template <int NV>
__device__ __forceinline__ bool finish_partials(const float (&v)[NV], float* partial, int nblk, int blk,
                                                unsigned* ticket, float* sh, int* flag) {
#pragma unroll
  for (int e = 0; e < NV; e++) {
    const float s = pcnn::wave_sum(v[e]);
    if (pcnn::lane_id() == 0) sh[(threadIdx.x >> 6) * NV + e] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    float s = 0.f;
    for (int w = 0; w < kBlk / 64; w++) s += sh[w * NV + threadIdx.x];
    partial[(size_t)blk * NV + threadIdx.x] = s;
  }
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) *flag = atomicAdd(ticket, 1u) == (unsigned)(nblk - 1);
  __syncthreads();
  if (!*flag) return false;
  __threadfence();
  if (threadIdx.x < NV) {  // totals -> sh[0, NV)
    float s = 0.f;
    s = ordered_sum_strided(partial + threadIdx.x, nblk, NV);
    sh[threadIdx.x] = s;
  }
  if (threadIdx.x == 0) *ticket = 0u;
  __syncthreads();
  return true;
}

// translation re-centring of solveICP for L objects (grid: segments x objects)
__global__ void __launch_bounds__(kBlk) k_icp_center(const float* __restrict__ live, const int32_t* __restrict__ label,
                                                     const int32_t* __restrict__ obj_ids,
                                                     const float* __restrict__ vertmap, const float* __restrict__ pred_v,
                                                     const float* __restrict__ pred_n, int HW, float max_error,
                                                     const float* __restrict__ pose_in, float* __restrict__ partial,
                                                     unsigned* __restrict__ tickets, float* __restrict__ out,
                                                     float* __restrict__ pose_out) {
  __shared__ float sh[(kBlk / 64) * 4];
  __shared__ int flag;
  const int l = blockIdx.y, seg = blockIdx.x, nblk = gridDim.x;
  const int obj = obj_ids[l];
  const float* lv = live + (size_t)l * HW * 3;
  const float* vm = vertmap + (size_t)l * HW * 3;
  const float* pv = pred_v + (size_t)l * HW * 4;
  const float* pn = pred_n + (size_t)l * HW * 4;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = threadIdx.x; i < kSeg; i += kBlk) {
    const int j = seg * kSeg + i;
    if (j >= HW || label[j] != obj) continue;
    const float d2 = lv[(size_t)j * 3 + 2];
    if (!(d2 > 0.f)) continue;
    const float mx = vm[(size_t)j * 3 + 0];
    const float mxr = mx - roundf(mx);  // the class offset dropped; std::round = half away from zero
    const float vy = vm[(size_t)j * 3 + 1], vz = vm[(size_t)j * 3 + 2];
    if (isnan(mxr) || isnan(vy) || isnan(vz)) continue;
    const float d0 = lv[(size_t)j * 3 + 0], d1 = lv[(size_t)j * 3 + 1];
    const float* n = pn + (size_t)j * 4;
    const float* p = pv + (size_t)j * 4;
    const float e = n[0] * (d0 - p[0]) + n[1] * (d1 - p[1]) + n[2] * (d2 - p[2]);
    if (fabsf(e) < max_error) {
      v[0] += d0 - mxr;
      v[1] += d1 - vy;
      v[2] += d2 - vz;
      v[3] += 1.f;
    }
  }
  if (!finish_partials<4>(v, partial + (size_t)l * nblk * 4, nblk, seg, tickets + l, sh, &flag)) return;
  if (threadIdx.x == 0) {
    const float c = sh[3];
    const float Tx = c > 0.f ? sh[0] / c : 0.f, Ty = c > 0.f ? sh[1] / c : 0.f, Tz = c > 0.f ? sh[2] / c : 0.f;
    float* o = out + (size_t)l * 4;
    o[0] = Tx; o[1] = Ty; o[2] = Tz; o[3] = c;
    if (pose_in && pose_out) {  // T_co.translation = (rx Tz, ry Tz, Tz) when c > 0 (:2207-2219)
      const float* P = pose_in + (size_t)l * 7;
      float* Q = pose_out + (size_t)l * 7;
      float rx = 0.f, ry = 0.f;
      if (P[6] != 0.f) {
        rx = P[4] / P[6];
        ry = P[5] / P[6];
      }
      for (int e = 0; e < 4; e++) Q[e] = P[e];
      Q[4] = c > 0.f ? rx * Tz : P[4];
      Q[5] = c > 0.f ? ry * Tz : P[5];
      Q[6] = c > 0.f ? Tz : P[6];
    }
  }
}

// optEnergy for K poses over the object's pixels (grid: segments x poses)
// (batched form: pose k belongs to problem (pose_obj[k], live map pose_live[k],
// rendered vertices pose_pv[k]); NULL index arrays = one problem for all K)
__global__ void __launch_bounds__(kBlk) k_pose_energy(const float* __restrict__ live_all,
                                                      const int32_t* __restrict__ label, int obj0,
                                                      const float* __restrict__ pv_all, int HW, float znear,
                                                      float zfar, const float* __restrict__ poses,
                                                      float* __restrict__ partial, unsigned* __restrict__ tickets,
                                                      float* __restrict__ energy, const int32_t* __restrict__ pose_obj,
                                                      const int32_t* __restrict__ pose_live,
                                                      const int32_t* __restrict__ pose_pv) {
  __shared__ float sh[(kBlk / 64) * 2];
  __shared__ int flag;
  const int k = blockIdx.y, seg = blockIdx.x, nblk = gridDim.x;
  const int obj = pose_obj ? pose_obj[k] : obj0;
  const float* __restrict__ live = live_all + (pose_live ? (size_t)pose_live[k] * HW * 3 : 0);
  const float* __restrict__ pred_v = pv_all + (pose_pv ? (size_t)pose_pv[k] * HW * 4 : 0);
  const float* P = poses + (size_t)k * 7;
  const float qn = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
  const Quat q = {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
  float v[2] = {0.f, 0.f};
  for (int i = threadIdx.x; i < kSeg; i += kBlk) {
    const int j = seg * kSeg + i;
    if (j >= HW || label[j] != obj) continue;
    float p0, p1, p2;
    rotate(q, pred_v[(size_t)j * 4 + 0], pred_v[(size_t)j * 4 + 1], pred_v[(size_t)j * 4 + 2], p0, p1, p2);
    p0 = p0 + P[4];
    p1 = p1 + P[5];
    p2 = p2 + P[6];
    const float l0 = live[(size_t)j * 3 + 0], l1 = live[(size_t)j * 3 + 1], l2 = live[(size_t)j * 3 + 2];
    if (!isnan(p0) && !isnan(p1) && !isnan(p2) && l2 > znear && l2 < zfar && p2 > znear && p2 < zfar) {
      const float dx = p0 - l0, dy = p1 - l1, dz = p2 - l2;
      v[0] += sqrtf(dx * dx + dy * dy + dz * dz);
      v[1] += 1.f;
    }
  }
  if (!finish_partials<2>(v, partial + (size_t)k * nblk * 2, nblk, seg, tickets + k, sh, &flag)) return;
  if (threadIdx.x == 0) energy[k] = sh[1] > 0.f ? sh[0] / sh[1] : 0.f;
}


// ---------------------------------------------------------------------------
// SegICP hypothesis score (synthesize.cpp:2288-2330).  The object's pixels
// with depth > 0 and a finite rendered vertmap give, in raster order, the
// model points (canonical vertmap, class offset dropped) and the depth points
// (live vertices).  For hypothesis j every transformed model point takes its
// nearest depth point within 1 cm (squared distance < 1e-4: FLANN's radius
// test; ties -> the lowest index) and flags it; score_j = distinct flagged
// depth points / model points.  The reference's order of flagging (an OpenMP
// race) does not change the count.
__device__ __forceinline__ bool score_pick(const float* __restrict__ live, const int32_t* __restrict__ label, int obj,
                                           const float* __restrict__ vertmap, int j) {
  if (label[j] != obj || !(live[(size_t)j * 3 + 2] > 0.f)) return false;
  const float mx = vertmap[(size_t)j * 3 + 0];
  return !isnan(mx - roundf(mx)) && !isnan(vertmap[(size_t)j * 3 + 1]) && !isnan(vertmap[(size_t)j * 3 + 2]);
}

__global__ void __launch_bounds__(kBlk) k_score_count(const float* __restrict__ live, const int32_t* __restrict__ label,
                                                      int obj, const float* __restrict__ vertmap, int HW, int nseg,
                                                      int32_t* __restrict__ cnt) {
  __shared__ int sh[kBlk / 64];
  int c = 0;
  for (int i = threadIdx.x; i < kSeg; i += kBlk) {
    const int j = blockIdx.x * kSeg + i;
    if (j < HW && score_pick(live, label, obj, vertmap, j)) c++;
  }
  c = block_sum_int<kBlk>(c, sh);
  if (threadIdx.x == 0) cnt[blockIdx.x] = c;
}

__global__ void __launch_bounds__(kBlk) k_score_scatter(const float* __restrict__ live,
                                                        const int32_t* __restrict__ label, int obj,
                                                        const float* __restrict__ vertmap, int HW, int nseg,
                                                        const int32_t* __restrict__ cnt, float4* __restrict__ model,
                                                        float4* __restrict__ dpts) {
  __shared__ int sh[kBlk / 64];
  __shared__ int wc[kBlk / 64];
  int o = 0;
  for (int s = threadIdx.x; s < (int)blockIdx.x; s += kBlk) o += cnt[s];
  int off = block_sum_int<kBlk>(o, sh);
  const int wave = threadIdx.x >> 6;
  for (int i0 = 0; i0 < kSeg; i0 += kBlk) {
    const int j = blockIdx.x * kSeg + i0 + threadIdx.x;
    const bool ok = j < HW && score_pick(live, label, obj, vertmap, j);
    const uint64_t m = __ballot(ok);
    if (pcnn::lane_id() == 0) wc[wave] = __popcll(m);
    __syncthreads();
    int base = off;
    for (int w = 0; w < wave; w++) base += wc[w];
    if (ok) {
      const int r = base + __popcll(m & pcnn::lanemask_lt());
      const float mx = vertmap[(size_t)j * 3 + 0];
      model[r] = make_float4(mx - roundf(mx), vertmap[(size_t)j * 3 + 1], vertmap[(size_t)j * 3 + 2], 0.f);
      dpts[r] = make_float4(live[(size_t)j * 3 + 0], live[(size_t)j * 3 + 1], live[(size_t)j * 3 + 2], 0.f);
    }
    for (int w = 0; w < kBlk / 64; w++) off += wc[w];
    __syncthreads();
  }
}

// Nearest depth point within the radius through a uniform grid (advisor
// finding: the brute-force M x M scan grows with the square of the object's
// pixel count).  Cells of edge s = 0.5005 r: a point closer than r to q
// differs from it by < 1.998 cells per axis (cell coordinates from double
// products, whose rounding is far below the margin for any |coordinate| <
// 10^7 m), so it lies within 2 cells of q's.  Cells hash into kGridBuckets
// buckets (counting sort of the depth-point indices); the query visits rings
// of cells outward and stops when the next ring cannot hold a point as close
// as its best.  Every point of every bucket visited is tested with the brute
// force's exact arithmetic, so the result -- the smallest squared distance
// < r^2, ties to the lowest index -- is the same (a hash collision only adds
// candidates; a bucket visited twice changes nothing).
constexpr int kGridBuckets = 1 << 17;

__device__ __forceinline__ bool grid_cell(float x, float y, float z, double inv_s, int& cx, int& cy, int& cz) {
  // in double: the product's rounding stays far below the 0.001-cell margin
  const double fx = floor((double)x * inv_s), fy = floor((double)y * inv_s), fz = floor((double)z * inv_s);
  if (!(fabs(fx) < 1e9 && fabs(fy) < 1e9 && fabs(fz) < 1e9)) return false;  // NaN / inf (never within r)
  cx = (int)fx;
  cy = (int)fy;
  cz = (int)fz;
  return true;
}

__device__ __forceinline__ int grid_bucket(int cx, int cy, int cz) {
  return (int)(((unsigned)cx * 73856093u ^ (unsigned)cy * 19349663u ^ (unsigned)cz * 83492791u) &
               (unsigned)(kGridBuckets - 1));
}

__device__ __forceinline__ int score_m(const int32_t* __restrict__ cnt, int nseg, int* ish) {
  int c = 0;
  for (int s = threadIdx.x; s < nseg; s += kBlk) c += cnt[s];
  return block_sum_int<kBlk>(c, ish);
}

// depth point -> bucket count (points outside the grid's range go nowhere:
// no query can be within r of them)
__global__ void __launch_bounds__(kBlk) k_grid_count(const float4* __restrict__ dpts, const int32_t* __restrict__ cnt,
                                                     int nseg, double inv_s, int32_t* __restrict__ bcount,
                                                     int32_t* __restrict__ bucket_of, int32_t* __restrict__ Mdev) {
  __shared__ int ish[kBlk / 64];
  const int M = score_m(cnt, nseg, ish);
  if (blockIdx.x == 0 && threadIdx.x == 0) *Mdev = M;  // the point count, for the launches after this one
  const int i = blockIdx.x * kBlk + threadIdx.x;
  if ((int)blockIdx.x * kBlk >= M || i >= M) return;
  const float4 d = dpts[i];
  int cx, cy, cz;
  int b = -1;
  if (grid_cell(d.x, d.y, d.z, inv_s, cx, cy, cz)) {
    b = grid_bucket(cx, cy, cz);
    atomicAdd(bcount + b, 1);
  }
  bucket_of[i] = b;
}

// exclusive scan of the bucket counts: start[b], start[NB] = total; cursor =
// start.  Two passes over kGridScanBlocks workgroups of 1024 buckets each (a
// single workgroup writing the 1 MB of starts and cursors took 110 us): the
// per-workgroup totals, then each workgroup adds the totals before it to a
// local scan of its own buckets.
constexpr int kGridScanBlocks = kGridBuckets / 1024;
__global__ void __launch_bounds__(256) k_grid_bsum(const int32_t* __restrict__ bcount, int32_t* __restrict__ bsum) {
  __shared__ int sh[4];
  const int4 v = ((const int4*)(bcount + (size_t)blockIdx.x * 1024))[threadIdx.x];
  const int s = block_sum_int<256>(v.x + v.y + v.z + v.w, sh);
  if (threadIdx.x == 0) bsum[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_grid_bscan(const int32_t* __restrict__ bcount,
                                                    const int32_t* __restrict__ bsum, int32_t* __restrict__ start,
                                                    int32_t* __restrict__ cursor) {
  __shared__ int sh[4], wsum[4];
  const int t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
  int pre = 0;  // totals of the workgroups before this one
  for (int i = t; i < (int)blockIdx.x; i += 256) pre += bsum[i];
  pre = block_sum_int<256>(pre, sh);
  const int4 v = ((const int4*)(bcount + (size_t)blockIdx.x * 1024))[t];
  const int mine = v.x + v.y + v.z + v.w;
  int inc = mine;  // inclusive wave scan of the 4-bucket sums
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int run = pre + inc - mine;
#pragma unroll
  for (int w = 0; w < 4; w++) run += w < wave ? wsum[w] : 0;
  int4 o;
  o.x = run;
  o.y = o.x + v.x;
  o.z = o.y + v.y;
  o.w = o.z + v.z;
  ((int4*)(start + (size_t)blockIdx.x * 1024))[t] = o;
  ((int4*)(cursor + (size_t)blockIdx.x * 1024))[t] = o;
  if (blockIdx.x == gridDim.x - 1 && t == 255) start[kGridBuckets] = o.w + v.w;
}

// the depth points in bucket order, each with its index (w: the int bits), so
// that the search reads a candidate with one load
__global__ void __launch_bounds__(kBlk) k_grid_fill(const int32_t* __restrict__ Mdev,
                                                    const float4* __restrict__ dpts,
                                                    const int32_t* __restrict__ bucket_of, int32_t* __restrict__ cursor,
                                                    float4* __restrict__ spts) {
  const int M = *Mdev;
  const int i = blockIdx.x * kBlk + threadIdx.x;
  if ((int)blockIdx.x * kBlk >= M || i >= M) return;
  const int b = bucket_of[i];
  if (b >= 0) {
    const float4 p = dpts[i];
    spts[atomicAdd(cursor + b, 1)] = make_float4(p.x, p.y, p.z, __int_as_float(i));
  }
}

// grid (query blocks, hypotheses): nearest depth point of each transformed
// model point, flagged when within the radius.  kNnLanes adjacent lanes share
// one query and split its cells (cell c of a ring to lane c % kNnLanes): a
// query is a chain of dependent bucket and point loads, and one lane per
// query left ~1 wave per SIMD to hide them.  The lanes' results merge as the
// lexicographic minimum of (squared distance, index) -- the sequential scan's
// first minimum -- and after each ring they share the smallest distance so
// far as the pruning bound.
#ifndef PCNN_NN_LANES
#define PCNN_NN_LANES 4
#endif
constexpr int kNnLanes = PCNN_NN_LANES;
__global__ void __launch_bounds__(kBlk) k_score_nn(const float4* __restrict__ model, const int32_t* __restrict__ Mdev,
                                                   const float* __restrict__ hyps, float r2, double inv_s,
                                                   const int32_t* __restrict__ start, const float4* __restrict__ spts,
                                                   uint8_t* __restrict__ flags, int cap) {
  constexpr int kQ = kBlk / kNnLanes;  // queries per workgroup
  const int M = *Mdev;
  const int h = blockIdx.y;
  const int sub = threadIdx.x % kNnLanes;
  const int q = blockIdx.x * kQ + threadIdx.x / kNnLanes;
  if ((int)blockIdx.x * kQ >= M || q >= M) return;  // a query's lanes leave together
  const float* P = hyps + (size_t)h * 7;
  const float qn = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
  const Quat qq = {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
  float x, y, z;
  const float4 m = model[q];
  rotate(qq, m.x, m.y, m.z, x, y, z);
  x = x + P[4];
  y = y + P[5];
  z = z + P[6];
  int cx, cy, cz;
  if (!grid_cell(x, y, z, inv_s, cx, cy, cz)) return;
  float best = r2;  // this lane's: strict, only squared distances < r2 qualify
  int bi = -1;
  float bound = r2;  // the query's smallest distance so far (all lanes), for pruning
  // rings of cells by Chebyshev distance d = 0, 1, 2 around q's cell (cells
  // of edge s = 0.5005 r: every point within r is at most 2 cells away).  A
  // cell is skipped when the squared distance from q to its box, less a 1e-5
  // relative margin (far above the fp32 distance's rounding), exceeds the
  // bound: no point in it can equal or beat the query's best.  Ring 2 is
  // skipped whole once (d - 1) s does.
  const double s_cell = 1.0 / inv_s;
  const double gx0 = (double)x - (double)cx * s_cell, gy0 = (double)y - (double)cy * s_cell,
               gz0 = (double)z - (double)cz * s_cell;  // q's offset inside its cell
  auto gap = [&](int o, double g) {  // distance from q to the cell o steps away along one axis
    return o > 0 ? (double)o * s_cell - g : (o < 0 ? g - (double)(o + 1) * s_cell : 0.0);
  };
  for (int d = 0; d <= 2; d++) {
    if (d >= 2 && (double)(d - 1) * s_cell * (d - 1) * s_cell * (1.0 - 1e-6) > (double)bound) break;
    int c = 0;
    for (int dz = -d; dz <= d; dz++)
      for (int dy = -d; dy <= d; dy++)
        for (int dx = -d; dx <= d; dx++) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != d) continue;
          if (c++ % kNnLanes != sub) continue;
          if (d > 0) {
            const double ax = fmax(gap(dx, gx0), 0.0), ay = fmax(gap(dy, gy0), 0.0), az = fmax(gap(dz, gz0), 0.0);
            if ((ax * ax + ay * ay + az * az) * (1.0 - 1e-5) > (double)bound) continue;
          }
          const int b = grid_bucket(cx + dx, cy + dy, cz + dz);
          const int e = start[b + 1];
          for (int k = start[b]; k < e; k++) {
            const float4 p = spts[k];
            const int i = __float_as_int(p.w);
            const float ex = x - p.x, ey = y - p.y, ez = z - p.z;
            const float d2 = ex * ex + ey * ey + ez * ez;
            if (d2 < best || (bi >= 0 && d2 == best && i < bi)) {  // the first minimum in index order
              best = d2;
              bi = i;
            }
          }
        }
    bound = fminf(bound, best);
#pragma unroll
    for (int o = 1; o < kNnLanes; o <<= 1) bound = fminf(bound, __shfl_xor(bound, o, kNnLanes));
  }
#pragma unroll
  for (int o = 1; o < kNnLanes; o <<= 1) {  // lexicographic minimum of (distance, index) over the query's lanes
    const float ob = __shfl_xor(best, o, kNnLanes);
    const int oi = __shfl_xor(bi, o, kNnLanes);
    if (oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi))) {
      best = ob;
      bi = oi;
    }
  }
  if (sub == 0 && bi >= 0) flags[(size_t)h * cap + bi] = 1;
}

// score per hypothesis: one workgroup per hypothesis counts its flags
__global__ void __launch_bounds__(1024) k_score_count_flags(const uint8_t* __restrict__ flags,
                                                            const int32_t* __restrict__ cnt, int nseg, int cap,
                                                            float* __restrict__ score) {
  __shared__ int ish[1024 / 64];
  int c = 0;
  for (int s = threadIdx.x; s < nseg; s += 1024) c += cnt[s];
  const int M = block_sum_int<1024>(c, ish);
  const int h = blockIdx.x;
  int f = 0;
  for (int i = threadIdx.x; i < M; i += 1024) f += flags[(size_t)h * cap + i];
  f = block_sum_int<1024>(f, ish);
  if (threadIdx.x == 0) score[h] = M > 0 ? (float)f / (float)M : 0.f;
}

// the first best hypothesis (one lane)
__global__ void k_score_choose(const float* __restrict__ score, const int32_t* __restrict__ cnt, int nseg, int J,
                               int32_t* __restrict__ choose) {
  if (threadIdx.x != 0) return;
  int M = 0;
  for (int s = 0; s < nseg; s++) M += cnt[s];
  float mx = -3.402823466e38f;
  int ch = -1;
  for (int h = 0; h < J; h++)
    if (score[h] > mx) {
      mx = score[h];
      ch = h;
    }
  *choose = M > 0 ? ch : 0;  // no depth point: hyps[0] (synthesize.cpp:2333-2334)
}

struct IcpWs {
  int32_t* cnt;
  float4* rec;
  float* acc;         // [2][N][8] accumulated update, by iteration parity
  float* partial;     // [2][N][kIcpSplitMax][kSys] per-slice systems, by iteration parity
};

inline IcpWs carve_icp(void* base, int N, int HW, size_t* bytes) {
  pcnn::Carve cv(base);
  IcpWs ws;
  const int nseg = (HW + kSeg - 1) / kSeg;
  ws.acc = cv.take<float>((size_t)2 * N * 8);
  ws.partial = cv.take<float>((size_t)2 * N * kIcpSplitMax * kSys);
  ws.cnt = cv.take<int32_t>((size_t)N * nseg);
  ws.rec = cv.take<float4>((size_t)N * HW * 2);
  if (bytes) *bytes = cv.off;
  return ws;
}

// partial sums + tickets of the segmented reductions
inline void carve_red(void* base, int L, int HW, int NV, float** partial, unsigned** tickets, size_t* bytes) {
  pcnn::Carve cv(base);
  const int nseg = (HW + kSeg - 1) / kSeg;
  *tickets = cv.take<unsigned>((size_t)L);
  *partial = cv.take<float>((size_t)L * nseg * NV);
  if (bytes) *bytes = cv.off;
}

}  // namespace pcnn_refine

using namespace pcnn_refine;

extern "C" int pcnn_icp_live_vertices(const uint16_t* depth, const int32_t* label, int H, int W,
                                      const int32_t* obj_ids, int L, float factor, float fx, float fy, float px,
                                      float py, float* out, void* stream) {
  PCNN_REQUIRE(depth && label && obj_ids && out && H > 0 && W > 0 && L > 0 && (H * W) % 4 == 0);
  const int HW = H * W;
  const int nb = (HW / 4 + kBlk - 1) / kBlk;
  hipLaunchKernelGGL(k_icp_live, dim3(nb, L), dim3(kBlk), 0, (hipStream_t)stream, depth, label, HW, W, obj_ids,
                     factor, fx, fy, px, py, out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" size_t pcnn_icp_workspace_size(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  size_t b = 0;
  carve_icp(nullptr, N, H * W, &b);
  return b + 256;
}

extern "C" int pcnn_icp(const float* live, int num_live, const int32_t* live_index, const float* pred_vertices,
                        const float* pred_normals, int N, int H, int W, float fx, float fy, float px, float py,
                        float znear, float zfar, float max_error, int iterations, const float* pose_in, float* update,
                        float* pose_out, float* systems, void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && pred_vertices && pred_normals && update && workspace && N > 0 && H > 0 && W > 0 &&
               num_live > 0 && (live_index || num_live >= N) && iterations >= 0 && (long)H * W * 2 * N < (1l << 31));
  size_t need = 0;
  carve_icp(nullptr, N, H * W, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  IcpWs ws = carve_icp(workspace, N, H * W, nullptr);
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_icp_count, dim3(nseg, N), dim3(kBlk), 0, st, pred_vertices, HW, znear, zfar, nseg, ws.cnt);
  hipLaunchKernelGGL(k_icp_scatter, dim3(nseg, N), dim3(kBlk), 0, st, pred_vertices, pred_normals, HW, znear, zfar,
                     nseg, ws.cnt, ws.rec);
  if (iterations == 0)
    hipLaunchKernelGGL(k_icp_identity, dim3((N + 63) / 64), dim3(64), 0, st, N, pose_in, update, pose_out);
  // about 512+ workgroups per launch: 1-2 records per lane for the usual footprints
  const int split = N >= 64 ? 8 : (512 / N > kIcpSplitMax ? kIcpSplitMax : (512 / N < 8 ? 8 : 512 / N));
  for (int it = 0; it < iterations; it++)
    hipLaunchKernelGGL(k_icp_step, dim3(split, N), dim3(kBlk), 0, st, ws.rec, ws.cnt, nseg, live, live_index,
                       num_live, H, W, fx, fy, px, py, znear, zfar, max_error, it, iterations, split, ws.acc,
                       ws.partial, systems);
  if (iterations > 0)
    hipLaunchKernelGGL(k_icp_finish, dim3(N), dim3(64), 0, st, N, iterations, split, ws.acc, ws.partial, pose_in,
                       update, pose_out, systems);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" size_t pcnn_icp_reduce_workspace_size(int L, int H, int W) {
  if (L <= 0 || H <= 0 || W <= 0) return 0;
  size_t b = 0;
  float* p;
  unsigned* t;
  carve_red(nullptr, L, H * W, 4, &p, &t, &b);
  return b + 256;
}

extern "C" int pcnn_icp_center(const float* live, const int32_t* label, const int32_t* obj_ids, int L,
                               const float* vertmap, const float* pred_vertices, const float* pred_normals, int H,
                               int W, float max_error, const float* pose_in, float* out, float* pose_out,
                               void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && label && obj_ids && vertmap && pred_vertices && pred_normals && out && workspace && L > 0 &&
               H > 0 && W > 0);
  size_t need = 0;
  float* partial;
  unsigned* tickets;
  carve_red(nullptr, L, H * W, 4, &partial, &tickets, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  carve_red(workspace, L, H * W, 4, &partial, &tickets, nullptr);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(tickets, 0, (size_t)L * sizeof(unsigned), st) != hipSuccess) return PCNN_EHIP;
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  hipLaunchKernelGGL(k_icp_center, dim3(nseg, L), dim3(kBlk), 0, st, live, label, obj_ids, vertmap, pred_vertices,
                     pred_normals, HW, max_error, pose_in, partial, tickets, out, pose_out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_pose_energy(const float* live, const int32_t* label, int obj, const float* pred_vertices, int H,
                                int W, float znear, float zfar, const float* poses, int K, float* energy,
                                void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && label && pred_vertices && poses && energy && workspace && K > 0 && H > 0 && W > 0);
  size_t need = 0;
  float* partial;
  unsigned* tickets;
  carve_red(nullptr, K, H * W, 4, &partial, &tickets, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  carve_red(workspace, K, H * W, 4, &partial, &tickets, nullptr);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(tickets, 0, (size_t)K * sizeof(unsigned), st) != hipSuccess) return PCNN_EHIP;
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  hipLaunchKernelGGL(k_pose_energy, dim3(nseg, K), dim3(kBlk), 0, st, live, label, obj, pred_vertices, HW, znear,
                     zfar, poses, partial, tickets, energy, (const int32_t*)nullptr, (const int32_t*)nullptr,
                     (const int32_t*)nullptr);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_pose_energy_batch(const float* live, int n_live, const int32_t* label, const float* pred_vertices,
                                      int n_pv, int H, int W, float znear, float zfar, const float* poses, int K,
                                      const int32_t* pose_obj, const int32_t* pose_live, const int32_t* pose_pv,
                                      float* energy, void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && label && pred_vertices && poses && energy && workspace && pose_obj && pose_live && pose_pv &&
               K > 0 && H > 0 && W > 0 && n_live > 0 && n_pv > 0);
  size_t need = 0;
  float* partial;
  unsigned* tickets;
  carve_red(nullptr, K, H * W, 4, &partial, &tickets, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  carve_red(workspace, K, H * W, 4, &partial, &tickets, nullptr);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(tickets, 0, (size_t)K * sizeof(unsigned), st) != hipSuccess) return PCNN_EHIP;
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  hipLaunchKernelGGL(k_pose_energy, dim3(nseg, K), dim3(kBlk), 0, st, live, label, 0, pred_vertices, HW, znear, zfar,
                     poses, partial, tickets, energy, pose_obj, pose_live, pose_pv);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" size_t pcnn_icp_score_workspace_size(int J, int H, int W) {
  if (J <= 0 || H <= 0 || W <= 0) return 0;
  pcnn::Carve cv(nullptr);
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  cv.take<int32_t>(nseg);
  cv.take<float4>((size_t)HW);
  cv.take<float4>((size_t)HW);
  cv.take<uint8_t>((size_t)J * HW);
  cv.take<int32_t>((size_t)kGridBuckets);      // bucket counts
  cv.take<int32_t>((size_t)kGridBuckets + 1);  // bucket starts
  cv.take<int32_t>((size_t)kGridBuckets);      // fill cursors
  cv.take<int32_t>((size_t)kGridScanBlocks + 1);  // bucket-scan workgroup totals, the point count
  cv.take<int32_t>((size_t)HW);                // bucket of each depth point
  cv.take<float4>((size_t)HW);                 // depth points (+ index) by bucket
  return cv.off + 256;
}

extern "C" int pcnn_icp_score(const float* live, const int32_t* label, int obj, const float* vertmap, int H, int W,
                              const float* hyps, int J, float radius, float* score, int32_t* choose, void* workspace,
                              size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && label && vertmap && hyps && score && choose && workspace && J > 0 && J <= 64 && H > 0 &&
               W > 0);
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  pcnn::Carve cv(workspace);
  int32_t* cnt = cv.take<int32_t>(nseg);
  float4* model = cv.take<float4>((size_t)HW);
  float4* dpts = cv.take<float4>((size_t)HW);
  uint8_t* flags = cv.take<uint8_t>((size_t)J * HW);
  int32_t* bcount = cv.take<int32_t>((size_t)kGridBuckets);
  int32_t* bstart = cv.take<int32_t>((size_t)kGridBuckets + 1);
  int32_t* cursor = cv.take<int32_t>((size_t)kGridBuckets);
  int32_t* bsum = cv.take<int32_t>((size_t)kGridScanBlocks + 1);
  int32_t* Mdev = bsum + kGridScanBlocks;
  int32_t* bucket_of = cv.take<int32_t>((size_t)HW);
  float4* spts = cv.take<float4>((size_t)HW);
  if (workspace_bytes < cv.off) return PCNN_ECAPACITY;
  PCNN_REQUIRE(radius > 0.f && radius < 1e6f);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(flags, 0, (size_t)J * HW, st) != hipSuccess) return PCNN_EHIP;
  if (hipMemsetAsync(bcount, 0, (size_t)kGridBuckets * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  const double inv_s = 1.0 / ((double)radius * 0.5005);
  const unsigned qblocks = (unsigned)((HW + kBlk - 1) / kBlk);
  hipLaunchKernelGGL(k_score_count, dim3(nseg), dim3(kBlk), 0, st, live, label, obj, vertmap, HW, nseg, cnt);
  hipLaunchKernelGGL(k_score_scatter, dim3(nseg), dim3(kBlk), 0, st, live, label, obj, vertmap, HW, nseg, cnt, model,
                     dpts);
  hipLaunchKernelGGL(k_grid_count, dim3(qblocks), dim3(kBlk), 0, st, dpts, cnt, nseg, inv_s, bcount, bucket_of, Mdev);
  hipLaunchKernelGGL(k_grid_bsum, dim3(kGridScanBlocks), dim3(256), 0, st, bcount, bsum);
  hipLaunchKernelGGL(k_grid_bscan, dim3(kGridScanBlocks), dim3(256), 0, st, bcount, bsum, bstart, cursor);
  hipLaunchKernelGGL(k_grid_fill, dim3(qblocks), dim3(kBlk), 0, st, Mdev, dpts, bucket_of, cursor, spts);
  hipLaunchKernelGGL(k_score_nn, dim3(qblocks * kNnLanes, J), dim3(kBlk), 0, st, model, Mdev, hyps, radius * radius,
                     inv_s, bstart, spts, flags, HW);
  hipLaunchKernelGGL(k_score_count_flags, dim3(J), dim3(1024), 0, st, flags, cnt, nseg, HW, score);
  hipLaunchKernelGGL(k_score_choose, dim3(1), dim3(64), 0, st, score, cnt, nseg, J, choose);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

// ---------------------------------------------------------------------------
// Nelder-Mead on optEnergy, on the device (round 5).  solveICP's refinePose
// (synthesize.cpp:2221-2250 -> poseWithOpt :2529-2573, NLopt LN_NELDERMEAD,
// 7 parameters, bounds +-0.1 / +-0.01 / +-0.1, at most `iterations`
// evaluations of optEnergy :2476-2526) used to run as Python generators with
// one energy launch and one host read per simplex step.  Here:
//   k_rec_count / k_rec_scatter  the object's pixels whose live vertex lies in
//       the depth range (the pose-independent half of optEnergy's test), in
//       raster order, as (rendered vertex, live vertex) records per problem;
//   energy_rec  optEnergy of one pose over a problem's records by one
//       1024-thread workgroup, a fixed summation order (thread-strided float
//       sums, then a fixed wave / workgroup tree): k_energy_rec evaluates K
//       poses, and k_nm runs whole searches, one workgroup per problem, with
//       no host read until the end.  The search is the bounded Nelder-Mead of
//       posecnn_amd/synthesize/icp.py nelder_mead_steps, operation for
//       operation in double (NLopt is absent: its trajectory is unpinned), so
//       the device search and the host search over k_energy_rec give the
//       same bits.
namespace pcnn_refine {

constexpr int kNmThreads = 1024;
constexpr int kNmDim = 7;

__global__ void __launch_bounds__(kBlk) k_rec_count(const float* __restrict__ live_all, int n_live,
                                                    const int32_t* __restrict__ label, int HW, float znear, float zfar,
                                                    const int32_t* __restrict__ prob_obj,
                                                    const int32_t* __restrict__ prob_live, int nseg,
                                                    int32_t* __restrict__ segcnt) {
  __shared__ int sh[kBlk / 64];
  const int p = blockIdx.y, seg = blockIdx.x;
  const int obj = prob_obj[p], li = prob_live[p];
  const bool ok_live = li >= 0 && li < n_live;
  const float* __restrict__ live = live_all + (ok_live ? (size_t)li * HW * 3 : 0);
  int c = 0;
  for (int i = threadIdx.x; i < kSeg; i += kBlk) {
    const int j = seg * kSeg + i;
    if (ok_live && j < HW && label[j] == obj) {
      const float lz = live[(size_t)j * 3 + 2];
      c += (lz > znear && lz < zfar) ? 1 : 0;  // :2514
    }
  }
  c = block_sum_int<kBlk>(c, sh);
  if (threadIdx.x == 0) segcnt[(size_t)p * nseg + seg] = c;
}

__global__ void __launch_bounds__(kBlk) k_rec_scatter(const float* __restrict__ live_all, int n_live,
                                                      const int32_t* __restrict__ label,
                                                      const float* __restrict__ pv_all, int HW, float znear,
                                                      float zfar, const int32_t* __restrict__ prob_obj,
                                                      const int32_t* __restrict__ prob_live, int nseg,
                                                      const int32_t* __restrict__ segcnt, float* __restrict__ rec,
                                                      int32_t* __restrict__ count) {
  __shared__ int sh[kBlk / 64];
  __shared__ int wc[kBlk / 64];
  const int p = blockIdx.y, seg = blockIdx.x;
  const int obj = prob_obj[p], li = prob_live[p];
  const bool ok_live = li >= 0 && li < n_live;
  const float* __restrict__ live = live_all + (ok_live ? (size_t)li * HW * 3 : 0);
  const float* __restrict__ pv = pv_all + (size_t)p * HW * 4;
  const int32_t* sc = segcnt + (size_t)p * nseg;
  int o = 0, tot = 0;
  for (int s = threadIdx.x; s < nseg; s += kBlk) {
    o += s < seg ? sc[s] : 0;
    tot += sc[s];
  }
  int off = block_sum_int<kBlk>(o, sh);
  const int total = block_sum_int<kBlk>(tot, sh);
  if (seg == 0 && threadIdx.x == 0) count[p] = total;
  float* out = rec + (size_t)p * HW * 6;
  const int wave = threadIdx.x >> 6;
  for (int i0 = 0; i0 < kSeg; i0 += kBlk) {
    const int j = seg * kSeg + i0 + threadIdx.x;
    bool ok = false;
    if (ok_live && j < HW && label[j] == obj) {
      const float lz = live[(size_t)j * 3 + 2];
      ok = lz > znear && lz < zfar;
    }
    const uint64_t m = __ballot(ok);
    if (pcnn::lane_id() == 0) wc[wave] = __popcll(m);
    __syncthreads();
    int base = off;
    for (int w = 0; w < wave; w++) base += wc[w];
    if (ok) {
      float* r = out + (size_t)(base + __popcll(m & pcnn::lanemask_lt())) * 6;
      r[0] = pv[(size_t)j * 4 + 0];
      r[1] = pv[(size_t)j * 4 + 1];
      r[2] = pv[(size_t)j * 4 + 2];
      r[3] = live[(size_t)j * 3 + 0];
      r[4] = live[(size_t)j * 3 + 1];
      r[5] = live[(size_t)j * 3 + 2];
    }
    for (int w = 0; w < kBlk / 64; w++) off += wc[w];
    __syncthreads();
  }
}

// optEnergy (:2476-2526) of pose P (float, quaternion normalised as
// k_pose_energy does) over n records; every thread of a 1024-thread
// workgroup calls it and gets the value
// the record sums of virtual thread vt (of kNmThreads): records vt, vt +
// kNmThreads, ... in order, four records' loads issued per pass (the loop
// was bound by one record's load latency at a time; the order is unchanged)
__device__ __forceinline__ void rec_sums(const float* __restrict__ r, int n, const Quat& q, const float (&P)[7],
                                         float znear, float zfar, int vt, float& s, float& c) {
  s = 0.f;
  c = 0.f;
  auto term = [&](const float* x) {
    float p0, p1, p2;
    rotate(q, x[0], x[1], x[2], p0, p1, p2);
    p0 = p0 + P[4];
    p1 = p1 + P[5];
    p2 = p2 + P[6];
    if (!isnan(p0) && !isnan(p1) && !isnan(p2) && p2 > znear && p2 < zfar) {  // :2514 (the live half: records)
      const float dx = p0 - x[3], dy = p1 - x[4], dz = p2 - x[5];
      s += sqrtf(dx * dx + dy * dy + dz * dz);
      c += 1.f;
    }
  };
  int i = vt;
  for (; i + 3 * kNmThreads < n; i += 4 * kNmThreads) {
    float v[4][6];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int e = 0; e < 6; e++) v[u][e] = r[(size_t)(i + u * kNmThreads) * 6 + e];
#pragma unroll
    for (int u = 0; u < 4; u++) term(v[u]);
  }
  for (; i < n; i += kNmThreads) term(r + (size_t)i * 6);
}

__device__ __forceinline__ Quat rec_quat(const float (&P)[7]) {
  const float qn = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
  return {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
}

// optEnergy (:2476-2526) of pose P (float, quaternion normalised as
// k_pose_energy does) over n records; every thread of a 1024-thread
// workgroup calls it and gets the value
__device__ float energy_rec(const float* __restrict__ r, int n, const float (&P)[7], float znear, float zfar,
                            float* sh) {
  const Quat q = rec_quat(P);
  float s, c;
  rec_sums(r, n, q, P, znear, zfar, threadIdx.x, s, c);
  s = pcnn::wave_sum(s);
  c = pcnn::wave_sum(c);
  const int wave = threadIdx.x >> 6;
  if (pcnn::lane_id() == 0) {
    sh[2 * wave] = s;
    sh[2 * wave + 1] = c;
  }
  __syncthreads();
  float S = 0.f, Cn = 0.f;
  for (int w = 0; w < kNmThreads / 64; w++) {
    S += sh[2 * w];
    Cn += sh[2 * w + 1];
  }
  __syncthreads();
  return Cn > 0.f ? S / Cn : 0.f;  // distance /= c (:2520-2521)
}

__global__ void __launch_bounds__(kNmThreads) k_energy_rec(const float* __restrict__ rec,
                                                           const int32_t* __restrict__ count, int stride,
                                                           const float* __restrict__ poses,
                                                           const int32_t* __restrict__ pose_prob, float znear,
                                                           float zfar, float* __restrict__ energy) {
  __shared__ float sh[2 * kNmThreads / 64];
  const int k = blockIdx.x;
  const int p = pose_prob[k];
  float P[7];
  for (int e = 0; e < 7; e++) P[e] = poses[(size_t)k * 7 + e];
  const float v = energy_rec(rec + (size_t)p * stride * 6, count[p], P, znear, zfar, sh);
  if (threadIdx.x == 0) energy[k] = v;
}

// Bounded Nelder-Mead (icp.py nelder_mead_steps, in its operation order):
// simplex x0 + step_i e_i with step = min(0.25 (ub - lb), 0.75 (ub - x0),
// 0.75 (x0 - lb)); each iteration a stable sort, the centroid of the best n
// (a sequential sum / n), reflection, expansion, contraction (outside /
// inside), shrink toward the best; trial points clamped to the bounds; at
// most max_eval evaluations.  One workgroup per problem: thread 0 keeps the
// simplex in LDS, every thread evaluates.
// Arrive-and-wait of the G workgroups of one problem on its counter (thread 0
// of each): release the workgroup's partial sums, wait until every workgroup
// of the problem has arrived for this evaluation.  Bounded: a wait that never
// completes (not expected: the launch is cooperative) gives up and raises the
// problem's failure flag; a workgroup waiting while the flag is up gives up at
// once.  A workgroup whose wait fails leaves the search (the caller checks
// s_fail after its barrier), so every workgroup of the problem stops at its
// next barrier instead of running on with sums that were never written, and
// the problem reports nev = -1.
__device__ __forceinline__ bool coop_arrive_wait(uint32_t* bar, uint32_t target, uint32_t* fail) {
  __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t cur = __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  for (int it = 0; cur < target && it < (1 << 24); it++) {
    if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    __builtin_amdgcn_s_sleep(2);
    cur = __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (cur >= target) return true;
  __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return false;
}

// nev reported by workgroup 0 of problem p: -1 when a cross-workgroup wait of
// the problem gave up (its own or another workgroup's: results invalid)
__device__ __forceinline__ int nm_report(int nev, int s_fail, const uint32_t* fail, int p) {
  if (s_fail) return -1;
  if (fail && __hip_atomic_load(fail + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return -1;
  return nev;
}

// G workgroups per problem (G = 1: one 1024-thread workgroup; G > 1: the
// 1024 "virtual threads" of optEnergy's reduction split over G workgroups of
// kNmThreads / G, each running the same search).  Every evaluation's record
// sums are those of energy_rec -- virtual thread v sums records v, v + 1024,
// ... in order, each 64 of them fold by the same butterfly, the 16 wave sums
// add in order -- so the value is identical for every G; with G > 1 the wave
// sums cross workgroups through `part` (double-buffered by evaluation
// parity) and one arrive-and-wait per evaluation on the problem's counter.
template <int G>
__global__ void __launch_bounds__(kNmThreads / G) k_nm(const float* __restrict__ rec,
                                                       const int32_t* __restrict__ count, int stride,
                                                       const double* __restrict__ x0_all,
                                                       const double* __restrict__ lb_all,
                                                       const double* __restrict__ ub_all, int max_eval, float znear,
                                                       float zfar, double* __restrict__ x_out,
                                                       double* __restrict__ f_out, int32_t* __restrict__ nev_out,
                                                       float* __restrict__ part, uint32_t* __restrict__ bar,
                                                       uint32_t* __restrict__ fail) {
  constexpr int n = kNmDim;
  constexpr int kT = kNmThreads / G;
  __shared__ double pts[n + 1][n], vals[n + 1], lb[n], ub[n], xq[n], xr[n], cen[n];
  __shared__ double fres;
  __shared__ float sh[2 * kNmThreads / 64];
  __shared__ int s_fail;
  const int p = blockIdx.x / G, g = blockIdx.x % G, t = threadIdx.x;
  const float* r = rec + (size_t)p * stride * 6;
  const int nr = count[p];
  int ne = 0;  // evaluations so far (the same in every thread of every workgroup of the problem)
  if (t == 0) s_fail = 0;
  auto eval = [&]() -> double {  // every thread; the point is xq (LDS)
    __syncthreads();
    float P[7];
    for (int e = 0; e < n; e++) P[e] = (float)xq[e];  // the host path evaluates float32 points
    float v;
    if constexpr (G == 1) {
      v = energy_rec(r, nr, P, znear, zfar, sh);
    } else {
      const int vt = g * kT + t;
      const Quat q = rec_quat(P);
      float s_, c_;
      rec_sums(r, nr, q, P, znear, zfar, vt, s_, c_);
      s_ = pcnn::wave_sum(s_);
      c_ = pcnn::wave_sum(c_);
      float* pp = part + ((size_t)p * 2 + (ne & 1)) * (2 * kNmThreads / 64);
      if (pcnn::lane_id() == 0) {
        pp[2 * (vt >> 6)] = s_;
        pp[2 * (vt >> 6) + 1] = c_;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      if (t == 0 && !coop_arrive_wait(bar + p, (uint32_t)(ne + 1) * G, fail + p)) s_fail = 1;
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      float S = 0.f, Cn = 0.f;
      for (int w = 0; w < kNmThreads / 64; w++) {
        S += pp[2 * w];
        Cn += pp[2 * w + 1];
      }
      v = Cn > 0.f ? S / Cn : 0.f;  // distance /= c (:2520-2521)
    }
    ne++;
    return (double)v;
  };
  auto clampq = [&](int e, double v) { return fmin(fmax(v, lb[e]), ub[e]); };  // np.minimum(np.maximum(p, lb), ub)
  if (t == 0) {
    for (int e = 0; e < n; e++) {
      lb[e] = lb_all[(size_t)p * n + e];
      ub[e] = ub_all[(size_t)p * n + e];
      pts[0][e] = x0_all[(size_t)p * n + e];
    }
    for (int i = 0; i < n; i++) {
      const double x0 = pts[0][i];
      const double step = fmin(0.25 * (ub[i] - lb[i]), fmin(0.75 * (ub[i] - x0), 0.75 * (x0 - lb[i])));
      for (int e = 0; e < n; e++) pts[i + 1][e] = pts[0][e] + (e == i ? step : 0.0);
    }
  }
  for (int i = 0; i <= n && !s_fail; i++) {  // the initial simplex (one batch on the host: the same values)
    if (t == 0)
      for (int e = 0; e < n; e++) xq[e] = pts[i][e];
    const double v = eval();
    if (t == 0) vals[i] = v;
  }
  int nev = n + 1;
  // nev and s_fail (read after each evaluation's barrier) are identical in
  // every thread; a failed wait ends the search in every workgroup
  while (nev < max_eval && !s_fail) {
    if (t == 0) {
      for (int i = 1; i <= n; i++) {  // stable insertion sort (np.argsort kind="stable")
        for (int j = i; j > 0 && vals[j] < vals[j - 1]; j--) {
          const double tv = vals[j];
          vals[j] = vals[j - 1];
          vals[j - 1] = tv;
          for (int e = 0; e < n; e++) {
            const double tp = pts[j][e];
            pts[j][e] = pts[j - 1][e];
            pts[j - 1][e] = tp;
          }
        }
      }
      for (int e = 0; e < n; e++) {  // np.mean(pts[:-1], axis=0): rows added in order, then / n
        double s = pts[0][e];
        for (int i = 1; i < n; i++) s = s + pts[i][e];
        cen[e] = s / (double)n;
      }
      for (int e = 0; e < n; e++) {
        xr[e] = clampq(e, cen[e] + (cen[e] - pts[n][e]));
        xq[e] = xr[e];
      }
    }
    const double fr = eval();
    nev++;
    __syncthreads();
    const double v0 = vals[0], vn1 = vals[n - 1], vn = vals[n];
    if (fr < v0 && nev < max_eval) {
      if (t == 0)
        for (int e = 0; e < n; e++) xq[e] = clampq(e, cen[e] + 2.0 * (cen[e] - pts[n][e]));
      const double fe = eval();
      nev++;
      if (t == 0) {
        const bool take_e = fe < fr;
        for (int e = 0; e < n; e++) pts[n][e] = take_e ? xq[e] : xr[e];
        vals[n] = take_e ? fe : fr;
      }
    } else if (fr < vn1) {
      if (t == 0) {
        for (int e = 0; e < n; e++) pts[n][e] = xr[e];
        vals[n] = fr;
      }
    } else if (nev < max_eval) {
      if (t == 0)
        for (int e = 0; e < n; e++)
          xq[e] = fr >= vn ? clampq(e, cen[e] + 0.5 * (pts[n][e] - cen[e])) : clampq(e, cen[e] + 0.5 * (xr[e] - cen[e]));
      const double fc = eval();
      nev++;
      if (fc < fmin(fr, vn)) {
        if (t == 0) {
          for (int e = 0; e < n; e++) pts[n][e] = xq[e];
          vals[n] = fc;
        }
      } else {
        const int m = min(n, max_eval - nev);
        for (int i = 1; i <= m && !s_fail; i++) {  // shrink toward the best (one batch on the host)
          if (t == 0)
            for (int e = 0; e < n; e++) xq[e] = clampq(e, pts[0][e] + 0.5 * (pts[i][e] - pts[0][e]));
          const double fv = eval();
          if (t == 0) {
            for (int e = 0; e < n; e++) pts[i][e] = xq[e];
            vals[i] = fv;
          }
        }
        nev += m > 0 ? m : 0;
      }
    }
    __syncthreads();
  }
  if (t == 0 && g == 0) {
    int b = 0;
    for (int i = 1; i <= n; i++)
      if (vals[i] < vals[b]) b = i;  // np.argmin: the first minimum
    for (int e = 0; e < n; e++) x_out[(size_t)p * n + e] = pts[b][e];
    f_out[p] = vals[b];
    nev_out[p] = nm_report(nev, s_fail, fail, p);
  }
  (void)fres;
}

// The same search with speculative rounds: kNmSpecW workgroup groups per
// problem, each of G workgroups evaluating one point of a round.  A round
// evaluates, in one arrive-and-wait, every point the next step may need:
// reflection, expansion and both contractions of an iteration (the sequential
// search then takes them in its own order and counts only those it uses), up
// to kNmSpecW points of the initial simplex or of a shrink.  optEnergy is a
// pure function of the point, so the simplex, the evaluation count and the
// result are those of k_nm bit for bit; an iteration costs one round (plus
// the shrink's) instead of one to three.
constexpr int kNmSpecW = 4;
template <int G, int S>
__global__ void __launch_bounds__(kNmThreads / G) k_nm_spec(const float* __restrict__ rec,
                                                            const int32_t* __restrict__ count, int stride,
                                                            const double* __restrict__ x0_all,
                                                            const double* __restrict__ lb_all,
                                                            const double* __restrict__ ub_all, int max_eval,
                                                            float znear, float zfar, double* __restrict__ x_out,
                                                            double* __restrict__ f_out, int32_t* __restrict__ nev_out,
                                                            float* __restrict__ part, uint32_t* __restrict__ bar,
                                                            uint32_t* __restrict__ fail) {
  constexpr int n = kNmDim;
  constexpr int kT = kNmThreads / G;
  constexpr int kW = 2 * kNmThreads / 64;  // (sum, count) per virtual wave
  __shared__ double pts[n + 1][n], vals[n + 1], lb[n], ub[n], cen[n], xs[S][n], fs[S];
  __shared__ int s_fail;
  const int p = blockIdx.x / (G * S), sp = (blockIdx.x / G) % S, g = blockIdx.x % G, t = threadIdx.x;
  const float* r = rec + (size_t)p * stride * 6;
  const int nr = count[p];
  int rnd = 0;  // rounds so far (the same in every thread of every workgroup of the problem)
  if (t == 0) s_fail = 0;
  auto round = [&](int cnt) {  // evaluate xs[0 .. cnt) -> fs[0 .. cnt), every thread
    __syncthreads();
    float* slot = part + ((size_t)p * 2 + (rnd & 1)) * S * kW;
    if (sp < cnt) {
      float P[7];
      for (int e = 0; e < n; e++) P[e] = (float)xs[sp][e];  // the host path evaluates float32 points
      const int vt = g * kT + t;
      const Quat q = rec_quat(P);
      float a, c;
      rec_sums(r, nr, q, P, znear, zfar, vt, a, c);
      a = pcnn::wave_sum(a);
      c = pcnn::wave_sum(c);
      if (pcnn::lane_id() == 0) {
        slot[sp * kW + 2 * (vt >> 6)] = a;
        slot[sp * kW + 2 * (vt >> 6) + 1] = c;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (t == 0 && !coop_arrive_wait(bar + p, (uint32_t)(rnd + 1) * G * S, fail + p)) s_fail = 1;
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (t < cnt) {  // value k: the 16 wave sums in order, as energy_rec
      float S_ = 0.f, C_ = 0.f;
      for (int w = 0; w < kNmThreads / 64; w++) {
        S_ += slot[t * kW + 2 * w];
        C_ += slot[t * kW + 2 * w + 1];
      }
      fs[t] = (double)(C_ > 0.f ? S_ / C_ : 0.f);  // distance /= c (:2520-2521)
    }
    rnd++;
    __syncthreads();
  };
  auto clampq = [&](int e, double v) { return fmin(fmax(v, lb[e]), ub[e]); };
  if (t == 0) {
    for (int e = 0; e < n; e++) {
      lb[e] = lb_all[(size_t)p * n + e];
      ub[e] = ub_all[(size_t)p * n + e];
      pts[0][e] = x0_all[(size_t)p * n + e];
    }
    for (int i = 0; i < n; i++) {
      const double x0 = pts[0][i];
      const double step = fmin(0.25 * (ub[i] - lb[i]), fmin(0.75 * (ub[i] - x0), 0.75 * (x0 - lb[i])));
      for (int e = 0; e < n; e++) pts[i + 1][e] = pts[0][e] + (e == i ? step : 0.0);
    }
  }
  for (int i0 = 0; i0 <= n && !s_fail; i0 += S) {  // the initial simplex
    const int cnt = min(S, n + 1 - i0);
    if (t == 0)
      for (int k = 0; k < cnt; k++)
        for (int e = 0; e < n; e++) xs[k][e] = pts[i0 + k][e];
    round(cnt);
    if (t == 0)
      for (int k = 0; k < cnt; k++) vals[i0 + k] = fs[k];
  }
  int nev = n + 1;
  while (nev < max_eval && !s_fail) {  // nev and s_fail are identical in every thread (a failed wait ends all)
    __syncthreads();
    if (t == 0) {
      for (int i = 1; i <= n; i++) {  // stable insertion sort (np.argsort kind="stable")
        for (int j = i; j > 0 && vals[j] < vals[j - 1]; j--) {
          const double tv = vals[j];
          vals[j] = vals[j - 1];
          vals[j - 1] = tv;
          for (int e = 0; e < n; e++) {
            const double tp = pts[j][e];
            pts[j][e] = pts[j - 1][e];
            pts[j - 1][e] = tp;
          }
        }
      }
      for (int e = 0; e < n; e++) {  // np.mean(pts[:-1], axis=0): rows added in order, then / n
        double sm = pts[0][e];
        for (int i = 1; i < n; i++) sm = sm + pts[i][e];
        cen[e] = sm / (double)n;
      }
      for (int e = 0; e < n; e++) {
        const double xr = clampq(e, cen[e] + (cen[e] - pts[n][e]));
        xs[0][e] = xr;                                            // reflection
        xs[1][e] = clampq(e, cen[e] + 2.0 * (cen[e] - pts[n][e]));  // expansion
        xs[2][e] = clampq(e, cen[e] + 0.5 * (xr - cen[e]));        // outside contraction
        xs[3][e] = clampq(e, cen[e] + 0.5 * (pts[n][e] - cen[e]));  // inside contraction
      }
    }
    round(4);
    const double fr = fs[0];
    nev++;
    const double v0 = vals[0], vn1 = vals[n - 1], vn = vals[n];
    __syncthreads();  // every thread holds v0 / vn1 / vn before thread 0 updates the simplex
    if (fr < v0 && nev < max_eval) {
      nev++;
      if (t == 0) {
        const bool take_e = fs[1] < fr;
        for (int e = 0; e < n; e++) pts[n][e] = take_e ? xs[1][e] : xs[0][e];
        vals[n] = take_e ? fs[1] : fr;
      }
    } else if (fr < vn1) {
      if (t == 0) {
        for (int e = 0; e < n; e++) pts[n][e] = xs[0][e];
        vals[n] = fr;
      }
    } else if (nev < max_eval) {
      nev++;
      const int kc = fr >= vn ? 3 : 2;
      const double fc = fs[kc];
      if (fc < fmin(fr, vn)) {
        if (t == 0) {
          for (int e = 0; e < n; e++) pts[n][e] = xs[kc][e];
          vals[n] = fc;
        }
      } else {
        const int m = min(n, max_eval - nev);
        for (int i0 = 1; i0 <= m && !s_fail; i0 += S) {  // shrink toward the best
          const int cnt = min(S, m + 1 - i0);
          __syncthreads();
          if (t == 0)
            for (int k = 0; k < cnt; k++)
              for (int e = 0; e < n; e++) xs[k][e] = clampq(e, pts[0][e] + 0.5 * (pts[i0 + k][e] - pts[0][e]));
          round(cnt);
          if (t == 0)
            for (int k = 0; k < cnt; k++) {
              for (int e = 0; e < n; e++) pts[i0 + k][e] = xs[k][e];
              vals[i0 + k] = fs[k];
            }
        }
        nev += m > 0 ? m : 0;
      }
    }
  }
  __syncthreads();
  if (t == 0 && g == 0 && sp == 0) {
    int b = 0;
    for (int i = 1; i <= n; i++)
      if (vals[i] < vals[b]) b = i;  // np.argmin: the first minimum
    for (int e = 0; e < n; e++) x_out[(size_t)p * n + e] = pts[b][e];
    f_out[p] = vals[b];
    nev_out[p] = nm_report(nev, s_fail, fail, p);
  }
}

}  // namespace pcnn_refine

extern "C" size_t pcnn_energy_records_workspace_size(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return 256;
  const int nseg = (H * W + kSeg - 1) / kSeg;
  return (size_t)N * nseg * sizeof(int32_t) + 256;
}

extern "C" int pcnn_energy_records(const float* live, int n_live, const int32_t* label, const float* pred_vertices,
                                   int H, int W, float znear, float zfar, int N, const int32_t* prob_obj,
                                   const int32_t* prob_live, float* records, int32_t* counts, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(live && label && pred_vertices && prob_obj && prob_live && records && counts && workspace);
  PCNN_REQUIRE(N > 0 && H > 0 && W > 0 && n_live > 0 && (long)H * W < (1l << 30));
  const int HW = H * W, nseg = (HW + kSeg - 1) / kSeg;
  if (workspace_bytes < (size_t)N * nseg * sizeof(int32_t)) return PCNN_ECAPACITY;
  int32_t* segcnt = (int32_t*)workspace;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_rec_count, dim3(nseg, N), dim3(kBlk), 0, st, live, n_live, label, HW, znear, zfar, prob_obj,
                     prob_live, nseg, segcnt);
  hipLaunchKernelGGL(k_rec_scatter, dim3(nseg, N), dim3(kBlk), 0, st, live, n_live, label, pred_vertices, HW, znear,
                     zfar, prob_obj, prob_live, nseg, segcnt, records, counts);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_energy_rec(const float* records, const int32_t* counts, int stride, const float* poses,
                               const int32_t* pose_prob, int K, float znear, float zfar, float* energy, void* stream) {
  PCNN_REQUIRE(records && counts && poses && pose_prob && energy && K > 0 && stride > 0);
  hipLaunchKernelGGL(k_energy_rec, dim3(K), dim3(kNmThreads), 0, (hipStream_t)stream, records, counts, stride, poses,
                     pose_prob, znear, zfar, energy);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_nelder_mead_energy(const float* records, const int32_t* counts, int stride, int N,
                                       const double* x0, const double* lb, const double* ub, int max_eval,
                                       float znear, float zfar, double* x_out, double* f_out, int32_t* nev_out,
                                       void* stream) {
  PCNN_REQUIRE(records && counts && x0 && lb && ub && x_out && f_out && nev_out && N > 0 && stride > 0);
  // at least the initial simplex: NLopt's maxeval also counts it, and a
  // budget below n + 1 is refused rather than overrun
  PCNN_REQUIRE(max_eval >= pcnn_refine::kNmDim + 1 && max_eval <= (1 << 20));
  hipLaunchKernelGGL(k_nm<1>, dim3(N), dim3(kNmThreads), 0, (hipStream_t)stream, records, counts, stride, x0, lb,
                     ub, max_eval, znear, zfar, x_out, f_out, nev_out, nullptr, nullptr, nullptr);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

// The same searches with kNmCoop workgroups per problem (the evaluation's
// records spread over kNmCoop CUs), launched cooperatively so that the
// workgroups of a problem are resident together; bit-identical results.
constexpr int kNmCoop = 8;
constexpr int kNmSpecMaxN = 32;  // N x 8 x 4 workgroups of 128 threads: 1024 at N = 32

static inline size_t nm_part_bytes(int N) {  // per problem: 2 parities x kNmSpecW points x the wave sums
  return pcnn::align_up((size_t)N * 2 * kNmSpecW * (2 * kNmThreads / 64) * sizeof(float), 256);
}
extern "C" size_t pcnn_nelder_mead_energy_workspace_size(int N) {
  if (N <= 0) return 256;
  return nm_part_bytes(N) + 2 * (size_t)N * sizeof(uint32_t) + 256;  // + the arrival counters and failure flags
}

extern "C" int pcnn_nelder_mead_energy_coop_path(const float* records, const int32_t* counts, int stride, int N,
                                                 const double* x0, const double* lb, const double* ub, int max_eval,
                                                 float znear, float zfar, double* x_out, double* f_out,
                                                 int32_t* nev_out, void* workspace, size_t workspace_bytes,
                                                 int force_path, int32_t* path_out, void* stream) {
  PCNN_REQUIRE(records && counts && x0 && lb && ub && x_out && f_out && nev_out && N > 0 && stride > 0);
  PCNN_REQUIRE(max_eval >= pcnn_refine::kNmDim + 1 && max_eval <= (1 << 20) && N <= 128);
  PCNN_REQUIRE(force_path >= 0 && force_path <= 3);
  if (!workspace || workspace_bytes < pcnn_nelder_mead_energy_workspace_size(N)) return PCNN_ECAPACITY;
  float* part = (float*)workspace;
  uint32_t* bar = (uint32_t*)((char*)workspace + nm_part_bytes(N));
  uint32_t* fail = bar + N;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(bar, 0, 2 * (size_t)N * sizeof(uint32_t), st) != hipSuccess) return PCNN_EHIP;
  void* args[] = {(void*)&records, (void*)&counts, (void*)&stride, (void*)&x0, (void*)&lb, (void*)&ub,
                  (void*)&max_eval, (void*)&znear, (void*)&zfar, (void*)&x_out, (void*)&f_out, (void*)&nev_out,
                  (void*)&part, (void*)&bar, (void*)&fail};
  // speculative rounds while the N x kNmCoop x kNmSpecW workgroups fit the
  // chip at once (path 1); then one evaluation per round (2); then one
  // workgroup per problem (3).  force_path pins one (0: the first that
  // launches); path_out (host int, may be null) reports the one that ran.
  int path = 0;
  if ((force_path == 0 || force_path == 1) && N <= kNmSpecMaxN &&
      hipLaunchCooperativeKernel((const void*)k_nm_spec<kNmCoop, kNmSpecW>, dim3(N * kNmCoop * kNmSpecW),
                                 dim3(kNmThreads / kNmCoop), args, 0, st) == hipSuccess)
    path = 1;
  if (!path) (void)hipGetLastError();
  if (!path && (force_path == 0 || force_path == 2) &&
      hipLaunchCooperativeKernel((const void*)k_nm<kNmCoop>, dim3(N * kNmCoop), dim3(kNmThreads / kNmCoop), args, 0,
                                 st) == hipSuccess)
    path = 2;
  if (!path) (void)hipGetLastError();
  if (!path && (force_path == 0 || force_path == 3)) {  // the one-workgroup search (same bits)
    hipLaunchKernelGGL(k_nm<1>, dim3(N), dim3(kNmThreads), 0, st, records, counts, stride, x0, lb, ub, max_eval,
                       znear, zfar, x_out, f_out, nev_out, nullptr, nullptr, nullptr);
    path = 3;
  }
  if (path_out) *path_out = path;
  if (!path) return PCNN_EHIP;  // the forced path could not launch
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_nelder_mead_energy_coop(const float* records, const int32_t* counts, int stride, int N,
                                            const double* x0, const double* lb, const double* ub, int max_eval,
                                            float znear, float zfar, double* x_out, double* f_out, int32_t* nev_out,
                                            void* workspace, size_t workspace_bytes, void* stream) {
  return pcnn_nelder_mead_energy_coop_path(records, counts, stride, N, x0, lb, ub, max_eval, znear, zfar, x_out, f_out,
                                           nev_out, workspace, workspace_bytes, 0, nullptr, stream);
}
