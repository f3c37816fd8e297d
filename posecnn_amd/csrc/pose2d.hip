// RGB-only pose estimation: Synthesizer::estimatePose2D
// (lib/synthesize/synthesize.cpp:1571-1766, synthesizer.pyx:74-82, called from
// lib/fcn/test.py:1364 under cfg.TEST.VERTEX_REG_3D) -- preemptive RANSAC
// over 2-D / 3-D correspondences from an object-coordinate vertex map.
//
// The reference runs it on the host: 256 hypotheses sampled by OpenMP threads
// (4 random pixels of one object, P3P, a reprojection and box-area check),
// then 8 preemptive rounds of inlier counting over a growing random subset of
// the object's pixels (std::mt19937 + negative_binomial skips), each round
// keeping the better half.  Here:
//   k_p2d_colcount / k_p2d_scan / k_p2d_scatter  the per-class pixel lists in
//       the reference's column-major order (getLabels, :1010-1031): per-column
//       class counts, a per-class scan over columns, an ordered scatter;
//   k_p2d_objs: object_ids (classes with > 400 pixels, :1027) and the list
//       offsets, on the device: no host round trip anywhere in the call;
//   k_p2d_subset: the 8 rounds' pixel subsets of each object (countInliers2D,
//       :1183-1213 -- identical for every hypothesis of a round).  The
//       reference skips max(1, G) pixels, G ~ negative_binomial(1, p) =
//       geometric with p = maxPixels / N, drawn from a default-seeded
//       std::mt19937.  Here G is drawn from a Philox stream per (class, round)
//       by inverse CDF on exact double products (G = the largest k with
//       U < q^k, q = 1 - p): the same distribution, computed identically by
//       the oracle; one workgroup per (object, round) draws 1024 gaps at a
//       time and places them by a block scan (round 5; the earlier host
//       replay of mt19937 draws cost 5.6 of the 6.2 ms per frame and pinned
//       nothing, since the hypotheses already use Philox streams);
//   k_p2d_attempts / k_p2d_pick: the rejection-sampling loop (samplePoint2D
//       x 4, degeneracy tests, Grunert P3P in double, the reprojection and
//       getBB2D area checks) as independent attempts, each on its own Philox
//       stream: the first 32 attempts of every hypothesis run at once (one
//       lane each), then one lane per hypothesis keeps its first accepted
//       attempt (one wave per hypothesis: 64 further attempts at a time, the
//       first accepted in attempt order, if none of the 32 was);
//   k_p2d_collect / k_p2d_count / k_select_sum / k_p2d_finish: the 8 rounds
//       as launches: per round one workgroup per (surviving hypothesis,
//       object) counts inliers over the round's subset (double projections),
//       then one workgroup per object keeps the better half by a stable rank
//       sort; the survivor's pose is written in the reference's (3, 4, C)
//       layout.
// The reference's refinement steps are inert in this path (updateHyp3D on an
// empty 3-D inlier list, optEnergy2D divided by that list's size: NLopt keeps
// the start point) and are not run; the oracle (oracle/orc_pose2d.cpp)
// documents the same reading.
#include "pcnn_common.h"
#include <climits>
#include <algorithm>

namespace {

constexpr int kRounds = 8;       // <= 256 hypotheses halve to one in <= 8 rounds; refIt = 8 (:1601)
constexpr int kMaxHypBlock = 1024;
constexpr int kMaxHyp = 256;     // ransacIterations (:1601)
constexpr int kAttempts = 32;  // sampling attempts per hypothesis evaluated in one launch
constexpr int kAttRec = 17;    // attempt record: obj (-1 rejected), R (9), t (3), pixels (4)
constexpr int kCntChunk = 512;  // subset entries per count workgroup pass
constexpr int kCntZ = 16;       // count workgroups per hypothesis at most (partial counts, summed by k_select_sum)
// round r's count workgroups per hypothesis: the early rounds have many
// hypotheses and short subsets, the late ones few hypotheses and long subsets
inline int count_z(int r) { return std::min(kCntZ, 2 << r); }

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// attempt a of hypothesis h draws Philox4x32-10 blocks (draw / 4, h, tag, a),
// words in order; tags 'P2D' (estimatePose2D), 'P3D' / 'F3D' (estimatePose3D)
constexpr uint32_t kTagP2D = 0x50324400u, kTagP3D = 0x50334400u, kTagF3D = 0x46334400u;
struct Stream {
  uint32_t k0, k1, h, tag, a, ctr;
  int word;
  U4 buf;
  __device__ Stream(uint64_t seed, uint32_t hyp, uint32_t tg, uint32_t attempt)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), h(hyp), tag(tg), a(attempt), ctr(0), word(4), buf{0, 0, 0, 0} {}
  __device__ uint32_t next() {
    if (word == 4) {
      buf = philox(U4{ctr++, h, tag, a}, k0, k1);
      word = 0;
    }
    const uint32_t v = word == 0 ? buf.x : word == 1 ? buf.y : word == 2 ? buf.z : buf.w;
    word++;
    return v;
  }
  __device__ int uniform(int n) {  // [0, n) by rejection of the top 2^32 mod n values
    const uint32_t un = (uint32_t)n;
    const uint32_t lim = (uint32_t)(0x100000000ull - (0x100000000ull % un));
    uint32_t x;
    do { x = next(); } while (lim != 0 && x >= lim);
    return (int)(x % un);
  }
};

struct D3 { double x, y, z; };
__device__ __forceinline__ D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ D3 scl(double s, D3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 cross(D3 a, D3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double nrm(D3 a) { return sqrt(dot(a, a)); }

struct F3 { float x, y, z; };
struct Pose { double R[9], t[3]; };
struct Cam { double fx, fy, px, py; };

// cv::projectPoints, no distortion (cvProjectPoints2's operation order)
__device__ __forceinline__ void project(const Pose& P, D3 X, const Cam& k, double& u, double& v) {
  const double x = P.R[0] * X.x + P.R[1] * X.y + P.R[2] * X.z + P.t[0];
  const double y = P.R[3] * X.x + P.R[4] * X.y + P.R[5] * X.z + P.t[1];
  double z = P.R[6] * X.x + P.R[7] * X.y + P.R[8] * X.z + P.t[2];
  z = z != 0.0 ? 1.0 / z : 1.0;
  u = x * z * k.fx + k.px;
  v = y * z * k.fy + k.py;
}

// getMode3D (:1052-1071): undo the [0, 1] extent scaling of the object coordinate
__device__ __forceinline__ F3 mode3d(const float* __restrict__ vm, const float* __restrict__ ext, int C, int obj, int p) {
  const float* m = vm + (size_t)p * 3 * C + 3 * obj;
  float o[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float vmin = -ext[obj * 3 + i] / 2, vmax = ext[obj * 3 + i] / 2;
    const float a = (float)(1.0 / (double)(vmax - vmin));
    const float b = (float)(-1.0 * (double)vmin / (double)(vmax - vmin));
    o[i] = (m[i] - b) / a;
  }
  return {o[0], o[1], o[2]};
}

__device__ __forceinline__ double norm3f(F3 a, F3 b) {
  const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return sqrt((double)dx * dx + (double)dy * dy + (double)dz * dz);
}

__device__ __forceinline__ double point_line(F3 p1, F3 p2, F3 p3) {  // :1074-1080
  const F3 a{p2.x - p1.x, p2.y - p1.y, p2.z - p1.z}, b{p3.x - p1.x, p3.y - p1.y, p3.z - p1.z};
  const F3 c{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  return sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z) /
         sqrt((double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z);
}

// complex helpers for the Durand-Kerner iteration
struct Cx { double re, im; };
__device__ __forceinline__ Cx cadd(Cx a, Cx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ Cx csub(Cx a, Cx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ Cx cmul(Cx a, Cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ Cx cdiv(Cx a, Cx b) {
  const double d = b.re * b.re + b.im * b.im;
  return {(a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d};
}

// real roots of c4 v^4 + ... + c0 (Durand-Kerner, then Newton polish)
__device__ int quartic_roots(const double* c, double* out) {
  double mx = 0;
  for (int i = 0; i < 4; i++) mx = fmax(mx, fabs(c[i]));
  if (!(fabs(c[4]) > 1e-12 * mx)) return 0;
  double a[4];
  for (int i = 0; i < 4; i++) a[i] = c[i] / c[4];
  double bound = 1;
  for (int i = 0; i < 4; i++) bound = fmax(bound, 1 + fabs(a[i]));
  Cx z[4];
  Cx w{1, 0};
  const Cx sd{0.4, 0.9};
  for (int k = 0; k < 4; k++) {
    z[k] = {w.re * bound, w.im * bound};
    w = cmul(w, sd);
  }
  // up to 200 sweeps, stopping at the first sweep whose steps are all below
  // 1e-9 of their root (the oracle stops at the same sweep: identical IEEE
  // double operations on both sides); the Newton polish below finishes the
  // real roots.  Round 5: 1e-13 was never reached by 2/3 of the quartics
  // (clustered roots oscillate at 1e-13..1e-10), so most ran all 200 sweeps;
  // at 1e-9, 97 % stop within 20 with the same real roots on the test scenes
  // (oracle outputs identical)
  for (int it = 0; it < 200; it++) {
    double mstep = 0;
    for (int k = 0; k < 4; k++) {
      Cx den{1, 0};
      for (int j = 0; j < 4; j++)
        if (j != k) den = cmul(den, csub(z[k], z[j]));
      if (den.re == 0 && den.im == 0) continue;
      Cx p = cadd(z[k], Cx{a[3], 0});
      p = cadd(cmul(p, z[k]), Cx{a[2], 0});
      p = cadd(cmul(p, z[k]), Cx{a[1], 0});
      p = cadd(cmul(p, z[k]), Cx{a[0], 0});
      const Cx st = cdiv(p, den);
      z[k] = csub(z[k], st);
      mstep = fmax(mstep, (fabs(st.re) + fabs(st.im)) / (1 + fabs(z[k].re) + fabs(z[k].im)));
    }
    if (mstep < 1e-9) break;
  }
  int n = 0;
  for (int k = 0; k < 4; k++) {
    const double az = sqrt(z[k].re * z[k].re + z[k].im * z[k].im);
    if (!(fabs(z[k].im) <= 1e-6 * (1 + az))) continue;
    double x = z[k].re;
    for (int it = 0; it < 4; it++) {
      const double p = (((x + a[3]) * x + a[2]) * x + a[1]) * x + a[0];
      const double dp = ((4 * x + 3 * a[3]) * x + 2 * a[2]) * x + a[1];
      if (dp == 0) break;
      x -= p / dp;
    }
    out[n++] = x;
  }
  return n;
}

__device__ Pose triad(const D3* P, const D3* Q) {
  D3 e[3], f[3];
  {
    e[0] = scl(1.0 / nrm(sub(P[1], P[0])), sub(P[1], P[0]));
    D3 w = sub(P[2], P[0]);
    w = sub(w, scl(dot(w, e[0]), e[0]));
    e[1] = scl(1.0 / nrm(w), w);
    e[2] = cross(e[0], e[1]);
  }
  {
    f[0] = scl(1.0 / nrm(sub(Q[1], Q[0])), sub(Q[1], Q[0]));
    D3 w = sub(Q[2], Q[0]);
    w = sub(w, scl(dot(w, f[0]), f[0]));
    f[1] = scl(1.0 / nrm(w), w);
    f[2] = cross(f[0], f[1]);
  }
  Pose o;
  const double fe[3][3] = {{f[0].x, f[1].x, f[2].x}, {f[0].y, f[1].y, f[2].y}, {f[0].z, f[1].z, f[2].z}};
  const double ee[3][3] = {{e[0].x, e[1].x, e[2].x}, {e[0].y, e[1].y, e[2].y}, {e[0].z, e[1].z, e[2].z}};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) o.R[3 * r + c] = fe[r][0] * ee[c][0] + fe[r][1] * ee[c][1] + fe[r][2] * ee[c][2];
  const double rp0 = o.R[0] * P[0].x + o.R[1] * P[0].y + o.R[2] * P[0].z;
  const double rp1 = o.R[3] * P[0].x + o.R[4] * P[0].y + o.R[5] * P[0].z;
  const double rp2 = o.R[6] * P[0].x + o.R[7] * P[0].y + o.R[8] * P[0].z;
  o.t[0] = Q[0].x - rp0;
  o.t[1] = Q[0].y - rp1;
  o.t[2] = Q[0].z - rp2;
  return o;
}

__device__ void polymul(const double* a, int na, const double* b, int nb, double* out) {
  for (int i = 0; i < na + nb - 1; i++) out[i] = 0;
  for (int i = 0; i < na; i++)
    for (int j = 0; j < nb; j++) out[i + j] += a[i] * b[j];
}

// solvePnP(CV_P3P) on 4 correspondences (Grunert's P3P with points 0-2, the
// solution reprojecting point 3 closest), as the oracle restates it
__device__ bool p3p(const F3* X, const float (*m)[2], const Cam& k, Pose& best) {
  D3 P[4], j[4];
  for (int i = 0; i < 4; i++) {
    P[i] = {X[i].x, X[i].y, X[i].z};
    const D3 r{((double)m[i][0] - k.px) / k.fx, ((double)m[i][1] - k.py) / k.fy, 1.0};
    j[i] = scl(1.0 / nrm(r), r);
  }
  const double a = nrm(sub(P[1], P[2])), b = nrm(sub(P[0], P[2])), c = nrm(sub(P[0], P[1]));
  const double ca = dot(j[1], j[2]), cb = dot(j[0], j[2]), cg = dot(j[0], j[1]);
  const double a2 = a * a, b2 = b * b, c2 = c * c;
  if (!(b2 > 0)) return false;
  const double K1 = (a2 - c2) / b2, Kc = c2 / b2;
  const double Nv[3] = {1 + K1, -2 * K1 * cb, K1 - 1};
  const double Dv[2] = {2 * cg, -2 * ca};
  const double qv[3] = {1 - Kc, 2 * Kc * cb, -Kc};
  double NN[5], ND[4], DD[3], qDD[5];
  polymul(Nv, 3, Nv, 3, NN);
  polymul(Nv, 3, Dv, 2, ND);
  polymul(Dv, 2, Dv, 2, DD);
  polymul(qv, 3, DD, 3, qDD);
  double poly[5];
  for (int i = 0; i < 5; i++) poly[i] = NN[i] - 2 * cg * (i < 4 ? ND[i] : 0) + qDD[i];
  double roots[4];
  const int nr = quartic_roots(poly, roots);
  double best_err = -1;
  for (int r = 0; r < nr; r++) {
    const double v = roots[r];
    const double D = 2 * (cg - v * ca);
    if (fabs(D) < 1e-12) continue;
    const double u = ((K1 - 1) * v * v - 2 * K1 * cb * v + 1 + K1) / D;
    const double q = 1 + v * v - 2 * v * cb;
    if (!(q > 0) || !(u > 0) || !(v > 0)) continue;
    const double s1 = sqrt(b2 / q);
    const D3 Q[3] = {scl(s1, j[0]), scl(u * s1, j[1]), scl(v * s1, j[2])};
    const Pose cand = triad(P, Q);
    double pu, pv;
    project(cand, P[3], k, pu, pv);
    const double e = (pu - m[3][0]) * (pu - m[3][0]) + (pv - m[3][1]) * (pv - m[3][1]);
    if (!(e == e)) continue;
    if (best_err < 0 || e < best_err) {
      best_err = e;
      best = cand;
    }
  }
  return best_err >= 0;
}

__device__ __forceinline__ int f2i_sat(float f) {  // C++ float -> int, defined for every input
  if (f != f) return 0;
  if (f >= 2147483648.0f) return INT_MAX;
  if (f <= -2147483648.0f) return INT_MIN;
  return (int)f;
}

// getBB2D (detection.h:78-109) area
__device__ int bb_area(const Pose& P, const float* ext, int obj, const Cam& k, int W, int H) {
  const float e0 = ext[obj * 3] * 0.5f, e1 = ext[obj * 3 + 1] * 0.5f, e2 = ext[obj * 3 + 2] * 0.5f;
  int minX = W - 1, maxX = 0, minY = H - 1, maxY = 0;
  for (int i = 0; i < 8; i++) {  // getBB3D corner order (detection.h:53-61)
    const float cx = (i & 1) ? -e0 : e0, cy = (i & 2) ? -e1 : e1, cz = (i & 4) ? -e2 : e2;
    double u, v;
    project(P, D3{cx, cy, cz}, k, u, v);
    const float fu = (float)u, fv = (float)v;
    minX = f2i_sat(fminf((float)minX, fu));
    minY = f2i_sat(fminf((float)minY, fv));
    maxX = f2i_sat(fmaxf((float)maxX, fu));
    maxY = f2i_sat(fmaxf((float)maxY, fv));
  }
  minX = min(max(minX, 0), W - 1);
  maxX = min(max(maxX, 0), W - 1);
  minY = min(max(minY, 0), H - 1);
  maxY = min(max(maxY, 0), H - 1);
  return (maxX - minX + 1) * (maxY - minY + 1);
}

struct P2dWs {
  int32_t* colcnt;   // (C, W) class pixels per column
  int32_t* coloff;   // (C, W) exclusive scan over columns
  int32_t* count;    // (C)
  int32_t* lists;    // (H W) per-class pixel lists, column-major, classes concatenated
  int32_t* listoff;  // (C) list offsets (k_p2d_objs)
  int32_t* objs;     // (C) object ids (k_p2d_objs)
  int32_t* nobj;     // (1) number of objects (k_p2d_objs)
  int32_t* sub;      // subsets: indices into the class list; class c round r at kRounds listoff[c] + r count[c]
  int32_t* subcnt;   // (C, kRounds) subset sizes
  double* hyp;       // (n_hyp, 16): obj, R (9), t (3)
  double* att;       // (n_hyp, kAttempts, kAttRec) attempt records
  int32_t* rl;       // (C, kMaxHypBlock) surviving hypotheses per object, in rank order
  int32_t* rc;       // (C, kMaxHypBlock) their inlier counts of the last round
  int32_t* rm;       // (C) survivors per object
  int32_t* pcnt;     // (C, kMaxHypBlock, kCntZ) partial inlier counts of a round's count kernel
};

// one wave per column (4 per workgroup): 64 rows at a time, class counts by
// LDS atomics (integer adds: order-free, exact), C <= 64 counters per wave
__global__ void __launch_bounds__(256) k_p2d_colcount(const int32_t* __restrict__ label, int H, int W, int C,
                                                      int32_t* colcnt) {
  __shared__ int cc[4][64];
  const int lane = pcnn::lane_id(), wv = threadIdx.x >> 6;
  const int x = blockIdx.x * 4 + wv;
  cc[wv][lane] = 0;
  __syncthreads();
  if (x < W) {
    for (int y0 = 0; y0 < H; y0 += 64) {
      const int y = y0 + lane;
      const int c = y < H ? label[y * W + x] : -1;
      if (c >= 0 && c < C) atomicAdd(&cc[wv][c], 1);
    }
  }
  __syncthreads();
  if (x < W && lane < C) colcnt[lane * W + x] = cc[wv][lane];
}

__global__ void __launch_bounds__(1024) k_p2d_scan(const int32_t* __restrict__ colcnt, int W, int32_t* coloff,
                                                   int32_t* count) {
  __shared__ int part[1024];
  const int c = blockIdx.x;
  int carry = 0;
  for (int base = 0; base < W; base += 1024) {
    const int x = base + threadIdx.x;
    const int v = x < W ? colcnt[c * W + x] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
      const int add = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (x < W) coloff[c * W + x] = carry + part[threadIdx.x] - v;
    carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) count[c] = carry;
}

// object_ids and list offsets (getLabels, :1010-1031): classes c >= 1 with
// more than minArea = 400 pixels, ascending
__global__ void __launch_bounds__(64) k_p2d_objs(int C, P2dWs ws) {
  if (threadIdx.x != 0) return;
  int acc = 0, n = 0;
  for (int c = 0; c < C; c++) {
    ws.listoff[c] = acc;
    const int cnt = ws.count[c];
    acc += cnt;
    if (c >= 1 && (float)cnt > 400.0f) ws.objs[n++] = c;
  }
  *ws.nobj = n;
}

// the subset of round r (0-based; maxPixels = 1000 (r + 1)) of class c's
// list: indices 0 = s_0 < s_1 < ... < N with s_{j+1} = s_j + max(1, G_j)
// (countInliers2D's skip, :1210-1213), G_j geometric with success
// probability p = maxPixels / (float)N, drawn from the Philox4x32-10 block
// (j, c, 'SUB0' + r, 0) under key seed: U = (x 2^21 + (y >> 11) + 0.5) 2^-53
// in (0, 1) from its first two words, G = the largest k with U < q^k,
// q = 1 - p, the powers by repeated double products (the oracle restates
// the same operations).  p >= 1: every index.
__device__ __forceinline__ int p2d_gap(uint64_t seed, int c, int r, int j, double q) {
  const U4 b = philox(U4{(uint32_t)j, (uint32_t)c, 0x53554230u + (uint32_t)r, 0u}, (uint32_t)seed,
                      (uint32_t)(seed >> 32));
  const double U = ((double)b.x * 2097152.0 + (double)(b.y >> 11) + 0.5) * 0x1p-53;
  int k = 0;
  double t = q;
  while (t > U) {  // q^(k+1) > U: G > k; at most 53 ln 2 / -ln q steps
    k++;
    t = t * q;
  }
  return k > 1 ? k : 1;
}

// the gap walk of a class list without depth holes: 1024 gaps at a time,
// placed by a block scan (block-uniform control flow; wsum: 16 ints of LDS)
__device__ void subset_nohole(uint64_t seed, int c, int r, int N, double q, int* S, int* subcnt, int* wsum) {
  const int t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
  long carry = 0;  // s_{j0}
  for (int j0 = 0;; j0 += 1024) {
    const int g = p2d_gap(seed, c, r, j0 + t, q);
    int incl = g;  // block inclusive scan of the gaps
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const int y = __shfl_up(incl, k, 64);
      if (lane >= k) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    long wb = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
      if (w < wave) wb += wsum[w];
      tot += wsum[w];
    }
    const long pos = carry + wb + incl - g;  // s_{j0 + t}
    if (pos < N) S[j0 + t] = (int)pos;
    if (pos < N && pos + g >= N) *subcnt = j0 + t + 1;  // the last index below N
    __syncthreads();  // wsum is rewritten by the next chunk
    if (carry + tot >= N) break;  // block-uniform
    carry += tot;
  }
}

__global__ void __launch_bounds__(1024) k_p2d_subset(uint64_t seed, P2dWs ws) {
  __shared__ int wsum[16];
  const int c = blockIdx.x, r = blockIdx.y, t = threadIdx.x;
  const int N = ws.count[c];
  if (c == 0 || !((float)N > 400.0f)) return;  // not an object (block-uniform)
  int* S = ws.sub + (size_t)kRounds * ws.listoff[c] + (size_t)r * N;
  const int maxPixels = 1000 * (r + 1);
  const float rate = maxPixels / (float)N;  // :1191
  if (!(rate < 1)) {  // every pixel (:1212-1213)
    for (int i = t; i < N; i += blockDim.x) S[i] = i;
    if (t == 0) ws.subcnt[c * kRounds + r] = N;
    return;
  }
  subset_nohole(seed, c, r, N, 1.0 - (double)rate, S, ws.subcnt + c * kRounds + r, wsum);
}

// one wave per column: 64 rows at a time; the lanes of one class take their
// ranks by ballot (classes peeled one at a time, usually 1-3 per chunk), so
// each class list keeps the column's ascending row order
__global__ void __launch_bounds__(256) k_p2d_scatter(const int32_t* __restrict__ label, int H, int W, int C, P2dWs ws) {
  __shared__ int run[4][64];  // per wave: class -> pixels placed so far in this column
  const int lane = pcnn::lane_id(), wv = threadIdx.x >> 6;
  const int x = blockIdx.x * 4 + wv;
  run[wv][lane] = 0;
  __syncthreads();
  if (x >= W) return;
  for (int y0 = 0; y0 < H; y0 += 64) {
    const int y = y0 + lane;
    const int c = y < H ? label[y * W + x] : -1;
    bool pending = c >= 0 && c < C;
    for (uint64_t left = __ballot(pending); left; left = __ballot(pending)) {
      const int cl = __shfl(c, __ffsll((unsigned long long)left) - 1);
      const uint64_t m = __ballot(pending && c == cl);
      const int base = run[wv][cl];
      if (pending && c == cl) {
        ws.lists[ws.listoff[cl] + ws.coloff[cl * W + x] + base + __popcll(m & pcnn::lanemask_lt())] = y * W + x;
        pending = false;
      }
      if (lane == 0) run[wv][cl] = base + __popcll(m);
    }
  }
}

// One sampling attempt of :1616-1688 (samplePoint2D x 4, the degeneracy
// tests, P3P, the 10 px reprojection and getBB2D area checks) on attempt a's
// own stream; true with the hypothesis when it is accepted.
__device__ bool p2d_attempt(const float* __restrict__ vm, const float* __restrict__ ext, int H, int W, int C,
                            const Cam& k, uint64_t seed, int h, int a, int n_obj, const P2dWs& ws, int& obj_out,
                            int* px_out, Pose& P) {
  Stream rs(seed, (uint32_t)h, kTagP2D, (uint32_t)a);
  const int obj = ws.objs[rs.uniform(n_obj)];  // n_obj > 0
  const int* L = ws.lists + ws.listoff[obj];
  const int N = ws.count[obj];
  float m[4][2];
  F3 X[4];
  int px4[4], n = 0;
  for (int s = 0; s < 4; s++) {  // samplePoint2D (:1084-1104)
    const int idx = L[rs.uniform(N)];
    const float u = (float)(idx % W), v = (float)(idx / W);
    double md = -1;
    for (int q = 0; q < n; q++) {
      const float dx = m[q][0] - u, dy = m[q][1] - v;
      const double d = sqrt((double)dx * dx + (double)dy * dy);
      md = md < 0 ? d : fmin(md, d);
    }
    if (md > 0 && md < 10) return false;
    const F3 o = mode3d(vm, ext, C, obj, idx);
    if (o.x == 0 && o.y == 0 && o.z == 0) return false;
    md = -1;
    for (int q = 0; q < n; q++) {
      const double d = norm3f(X[q], o);
      md = md < 0 ? d : fmin(md, d);
    }
    if (md > 0 && md < 0.01) return false;
    m[n][0] = u;
    m[n][1] = v;
    X[n] = o;
    px4[n] = idx;
    n++;
  }
  if (point_line(X[0], X[1], X[2]) < 0.01 || point_line(X[0], X[1], X[3]) < 0.01 ||
      point_line(X[0], X[2], X[3]) < 0.01 || point_line(X[1], X[2], X[3]) < 0.01)
    return false;
  if (!p3p(X, m, k, P)) return false;
  for (int q = 0; q < 4; q++) {  // the 4 samples must reproject within 10 px (:1664-1672)
    double u, v;
    project(P, D3{X[q].x, X[q].y, X[q].z}, k, u, v);
    const float du = m[q][0] - (float)u, dv = m[q][1] - (float)v;
    if (!(sqrt((double)du * du + (double)dv * dv) < 10)) return false;
  }
  if ((float)bb_area(P, ext, obj, k, W, H) < 400.0f) return false;  // :1678-1680
  obj_out = obj;
  for (int i = 0; i < 4; i++) px_out[i] = px4[i];
  return true;
}

// ---------------------------------------------------------------------------
// estimatePose3D's pieces shared with the attempt kernels (synthesize.cpp:
// 1769-1965; the oracle, oracle/orc_pose2d.cpp orc_pose3d, restates the same
// operations in the same order).

struct AttArgs {  // the sampling attempt's inputs
  const float* vm;
  const float* ext;
  const float* eye;  // (H, W, 3) camera coordinates (estimatePose3D only)
  int H, W, C;
  Cam k;
  uint64_t seed;
};

__device__ __forceinline__ F3 eye_at(const float* __restrict__ eye, int p) {
  return {eye[(size_t)p * 3], eye[(size_t)p * 3 + 1], eye[(size_t)p * 3 + 2]};
}

// one-sided Jacobi SVD of a 3x3 (row-major): A = U diag(S) V^T, S descending;
// fixed pivot order (0,1), (0,2), (1,2), at most 16 sweeps; U's third column
// the cross product of the first two when the covariance has rank two
__device__ void svd3(const double* A, double* U, double* S, double* V) {
  double M[9], Vm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int i = 0; i < 9; i++) M[i] = A[i];
  for (int sweep = 0; sweep < 16; sweep++) {
    bool rot = false;
    for (int kk = 0; kk < 3; kk++) {
      const int p = kk == 2 ? 1 : 0, q = kk == 0 ? 1 : 2;
      double al = 0, be = 0, ga = 0;
      for (int r = 0; r < 3; r++) {
        al = al + M[r * 3 + p] * M[r * 3 + p];
        be = be + M[r * 3 + q] * M[r * 3 + q];
        ga = ga + M[r * 3 + p] * M[r * 3 + q];
      }
      if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
      const double zeta = (be - al) / (2.0 * ga);
      const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
      for (int r = 0; r < 3; r++) {
        const double mp = M[r * 3 + p], mq = M[r * 3 + q];
        M[r * 3 + p] = c * mp - s * mq;
        M[r * 3 + q] = s * mp + c * mq;
        const double vp = Vm[r * 3 + p], vq = Vm[r * 3 + q];
        Vm[r * 3 + p] = c * vp - s * vq;
        Vm[r * 3 + q] = s * vp + c * vq;
      }
      rot = true;
    }
    if (!rot) break;
  }
  double sv[3];
  for (int i = 0; i < 3; i++) {
    double a = 0;
    for (int r = 0; r < 3; r++) a = a + M[r * 3 + i] * M[r * 3 + i];
    sv[i] = sqrt(a);
  }
  // descending, stable (the oracle's insertion sort), as selects: no
  // dynamically indexed arrays, so everything stays in registers
  auto pick3 = [](const double* a, int i) { return i == 0 ? a[0] : i == 1 ? a[1] : a[2]; };
  int o0 = 0, o1 = 1, o2 = 2;
  if (pick3(sv, o1) > pick3(sv, o0)) { const int tmp = o0; o0 = o1; o1 = tmp; }
  if (pick3(sv, o2) > pick3(sv, o1)) {
    { const int tmp = o1; o1 = o2; o2 = tmp; }
    if (pick3(sv, o1) > pick3(sv, o0)) { const int tmp = o0; o0 = o1; o1 = tmp; }
  }
  const int o[3] = {o0, o1, o2};
#pragma unroll
  for (int kk = 0; kk < 3; kk++) {
    S[kk] = pick3(sv, o[kk]);
#pragma unroll
    for (int r = 0; r < 3; r++) {
      V[r * 3 + kk] = pick3(Vm + r * 3, o[kk]);
      U[r * 3 + kk] = S[kk] > 0 ? pick3(M + r * 3, o[kk]) / S[kk] : 0.0;
    }
  }
  if (!(S[2] > 1e-9 * S[0])) {
    U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
    U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
    U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
  }
}

__device__ __forceinline__ double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// calcRigidBodyTransform (Hypothesis.cpp:217-241) from the centroids and the
// covariance: R = V diag(1, 1, sign det(V U^T)) U^T, t = -R cA + cB
__device__ __forceinline__ Pose rigid_from_cov(const double* Hc, const double* cA, const double* cB) {
  double U[9], S[3], V[9];
  svd3(Hc, U, S, V);
  double VU[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) VU[r * 3 + c] = V[r * 3 + 0] * U[c * 3 + 0] + V[r * 3 + 1] * U[c * 3 + 1] + V[r * 3 + 2] * U[c * 3 + 2];
  const double sg = det3(VU) < 0 ? -1.0 : 1.0;
  Pose P;
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      P.R[r * 3 + c] = V[r * 3 + 0] * U[c * 3 + 0] + V[r * 3 + 1] * U[c * 3 + 1] + (V[r * 3 + 2] * sg) * U[c * 3 + 2];
  for (int r = 0; r < 3; r++) P.t[r] = -(P.R[r * 3 + 0] * cA[0] + P.R[r * 3 + 1] * cA[1] + P.R[r * 3 + 2] * cA[2]) + cB[r];
  return P;
}

// out of line for the 1024-thread k_p3d_update: only its thread 0 runs it,
// and inlined it would set the whole workgroup's register budget
__device__ __noinline__ Pose rigid_from_cov_ool(const double* Hc, const double* cA, const double* cB) {
  return rigid_from_cov(Hc, cA, cB);
}

// The fixed summation tree of a 1024-thread workgroup (the oracle's
// tree1024): leaf i = 0.0 + x_i (0 past n), each wave folds its 64 leaves by
// halving (p_i += p_{i + off}, off = 32 .. 1), then the 16 wave sums fold the
// same way (off = 8 .. 1).
// fold_small<n>: that tree over n <= 4 leaves held by one lane, zeros
// included (the additions of 0.0 matter only to the sign of a zero, kept
// anyway)
template <int n>
__device__ __forceinline__ double fold_small(const double* x) {
  double p[64];
#pragma unroll
  for (int l = 0; l < 64; l++) p[l] = l < n ? 0.0 + x[l] : 0.0;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int i = 0; i < off; i++) p[i] = p[i] + p[i + off];
  double w = p[0];
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) w = w + 0.0;  // the other 15 wave sums are zero
  return w;
}

// the in-wave half of the tree: the wave's sum on lane 0 (other lanes: partial)
template <class T>
__device__ __forceinline__ T wave_fold(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const T w = __shfl_down(v, off, 64);
    v = v + w;
  }
  return v;
}

// the cross-wave half: ws[16][K] wave sums (LDS, visible) -> the tree's total
template <class T, int K>
__device__ __forceinline__ T cross_fold(const T (*ws)[K], int k) {
  T w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = ws[i][k];
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1)
#pragma unroll
    for (int i = 0; i < off; i++) w[i] = w[i] + w[i + off];
  return w[0];
}

__device__ __forceinline__ D3 xform(const Pose& P, D3 p) {  // Hypothesis::transform
  return {P.R[0] * p.x + P.R[1] * p.y + P.R[2] * p.z + P.t[0], P.R[3] * p.x + P.R[4] * p.y + P.R[5] * p.z + P.t[1],
          P.R[6] * p.x + P.R[7] * p.y + P.R[8] * p.z + P.t[2]};
}

// One sampling attempt of :1814-1889: samplePoint3D x 3 (:1105-1134: depth
// hole, 1 cm camera / object spacing, empty prediction), the 3-point rigid
// transform, the 1 cm reconstruction check, getBB2D area >= 400
__device__ bool p3d_attempt(const AttArgs& A, int h, int a, int n_obj, const P2dWs& ws, int& obj_out, int* px_out,
                            Pose& P) {
  Stream rs(A.seed, (uint32_t)h, kTagP3D, (uint32_t)a);
  const int obj = ws.objs[rs.uniform(n_obj)];
  const int* L = ws.lists + ws.listoff[obj];
  const int N = ws.count[obj];
  F3 E[3], O[3];
  int n = 0;
  for (int s = 0; s < 3; s++) {
    const int idx = L[rs.uniform(N)];
    const F3 e = eye_at(A.eye, idx);
    if (e.z == 0) return false;
    double md = -1;
    for (int q = 0; q < n; q++) md = md < 0 ? norm3f(E[q], e) : fmin(md, norm3f(E[q], e));
    if (md > 0 && md < 0.01) return false;
    const F3 o = mode3d(A.vm, A.ext, A.C, obj, idx);
    if (o.x == 0 && o.y == 0 && o.z == 0) return false;
    md = -1;
    for (int q = 0; q < n; q++) md = md < 0 ? norm3f(O[q], o) : fmin(md, norm3f(O[q], o));
    if (md > 0 && md < 0.01) return false;
    E[n] = e;
    O[n] = o;
    px_out[n] = idx;
    n++;
  }
  const double inv = 1.0 / 3.0;
  double cA[3], cB[3], Hc[9];
  {
    double xa[3][3], xb[3][3];  // [coordinate][point]
    for (int q = 0; q < 3; q++) {
      xa[0][q] = O[q].x; xa[1][q] = O[q].y; xa[2][q] = O[q].z;
      xb[0][q] = E[q].x; xb[1][q] = E[q].y; xb[2][q] = E[q].z;
    }
    for (int r = 0; r < 3; r++) {
      cA[r] = fold_small<3>(xa[r]) * inv;
      cB[r] = fold_small<3>(xb[r]) * inv;
    }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        double pr[3];
        for (int q = 0; q < 3; q++) pr[q] = (xa[r][q] - cA[r]) * (xb[c][q] - cB[c]);
        Hc[r * 3 + c] = fold_small<3>(pr);
      }
  }
  P = rigid_from_cov(Hc, cA, cB);
  for (int q = 0; q < 3; q++) {  // :1859-1867
    const D3 b{E[q].x, E[q].y, E[q].z};
    if (!(nrm(sub(b, xform(P, D3{O[q].x, O[q].y, O[q].z}))) < 0.01)) return false;
  }
  if ((float)bb_area(P, A.ext, obj, A.k, A.W, A.H) < 400.0f) return false;  // :1877-1882
  obj_out = obj;
  return true;
}

// sin / cos / acos from + - * / sqrt only (the oracle's dsincos / dacos):
// quadrant reduction by a two-part pi/2, the fdlibm kernel polynomials; acos
// by the half-angle identity and 6 Newton steps on asin
__device__ void dsincos(double x, double& s, double& c) {
  const double n = floor(x * 0.63661977236758134308 + 0.5);
  const double y = (x - n * 1.57079632673412561417e+00) - n * 6.07710050650619224932e-11;
  const double z = y * y;
  const double ks = y + y * z * (-1.66666666666666324348e-01 + z * (8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 +
                        z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)))));
  const double kc = 1.0 - (0.5 * z - z * z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * (2.48015872894767294178e-05 +
                        z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11))))));
  const int q = ((int)n) & 3;
  s = q == 0 ? ks : q == 1 ? kc : q == 2 ? -ks : -kc;
  c = q == 0 ? kc : q == 1 ? -ks : q == 2 ? -kc : ks;
}

__device__ double dasin_small(double x) {
  double y = x;
  for (int i = 0; i < 6; i++) {
    double s, c;
    dsincos(y, s, c);
    y = y - (s - x) / c;
  }
  return y;
}

__device__ double dacos(double c) {
  if (c >= 0) return 2.0 * dasin_small(sqrt((1.0 - c) * 0.5));
  return 3.14159265358979311600 - 2.0 * dasin_small(sqrt((1.0 + c) * 0.5));
}

// cv::Rodrigues vector -> matrix
__device__ void rod_v2m(const double* r, double* R) {
  const double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < 2.220446049250313e-16) {
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  double s, c;
  dsincos(th, s, c);
  const double c1 = 1.0 - c, it = 1.0 / th;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  for (int i = 0; i < 9; i++) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

// cv::Rodrigues matrix -> vector (without cvRodrigues2's re-orthonormalisation)
__device__ void rod_m2v(const double* R, double* r) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double th = dacos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double t = (R[0] + 1) * 0.5;
      rx = sqrt(fmax(t, 0.));
      t = (R[4] + 1) * 0.5;
      ry = sqrt(fmax(t, 0.)) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5;
      rz = sqrt(fmax(t, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      th /= sqrt(rx * rx + ry * ry + rz * rz);
      rx *= th;
      ry *= th;
      rz *= th;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= th;
    rx *= vth;
    ry *= vth;
    rz *= vth;
  }
  r[0] = rx;
  r[1] = ry;
  r[2] = rz;
}

// The first kAttempts attempts of every hypothesis at once, one lane each:
// the reference's loop runs attempts until one is accepted, and attempts are
// independent (each its own stream), so they need not wait for each other.
// kDepth: estimatePose3D's attempt (3 pixels), else estimatePose2D's (4).
template <bool kDepth>
__device__ __forceinline__ bool attempt(const AttArgs& A, int h, int a, int n_obj, const P2dWs& ws, int& obj,
                                        int* px, Pose& P) {
  if constexpr (kDepth)
    return p3d_attempt(A, h, a, n_obj, ws, obj, px, P);
  else
    return p2d_attempt(A.vm, A.ext, A.H, A.W, A.C, A.k, A.seed, h, a, n_obj, ws, obj, px, P);
}

template <bool kDepth>
__global__ void __launch_bounds__(64) k_attempts(AttArgs A, int n_hyp, int T, P2dWs ws) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_obj = *ws.nobj;
  if (id >= n_hyp * T || n_obj == 0) return;
  const int h = id % n_hyp, a = id / n_hyp;
  double* rec = ws.att + (size_t)(h * T + a) * kAttRec;
  int obj, px4[4] = {-1, -1, -1, -1};
  Pose P;
  if (!attempt<kDepth>(A, h, a, n_obj, ws, obj, px4, P)) {
    rec[0] = -1;
    return;
  }
  rec[0] = obj;
  for (int i = 0; i < 9; i++) rec[1 + i] = P.R[i];
  for (int i = 0; i < 3; i++) rec[10 + i] = P.t[i];
  for (int i = 0; i < 4; i++) rec[13 + i] = px4[i];
}

// One wave per hypothesis: its first accepted attempt in attempt order --
// the batch above, then (rarely) 64 further attempts at a time, each lane
// one attempt, the lowest accepted lane kept -- written out as :1682-1686
// (:1884-1887) store it.  max_iter bounds the attempts (the reference:
// 10,000,000).
template <bool kDepth>
__global__ void __launch_bounds__(64) k_pick(AttArgs A, int n_hyp, int max_iter, int T, P2dWs ws,
                                             float* __restrict__ hyps_out, int32_t* __restrict__ hyp_px) {
  constexpr int kPx = kDepth ? 3 : 4;
  const int h = blockIdx.x, lane = pcnn::lane_id();
  if (h >= n_hyp) return;
  const int n_obj = *ws.nobj;
  // the batch: lane a < T reads attempt a's record; the first accepted one wins
  int a_hit = -1;
  {
    const bool acc = lane < T && n_obj > 0 && ws.att[(size_t)(h * T + lane) * kAttRec] >= 0;
    const uint64_t b = __ballot(acc);
    if (b) a_hit = __ffsll((unsigned long long)b) - 1;
  }
  int obj = -1, px4[4] = {-1, -1, -1, -1};
  Pose P;
  if (a_hit >= 0) {
    const double* rec = ws.att + (size_t)(h * T + a_hit) * kAttRec;
    obj = (int)rec[0];
    for (int i = 0; i < 9; i++) P.R[i] = rec[1 + i];
    for (int i = 0; i < 3; i++) P.t[i] = rec[10 + i];
    for (int i = 0; i < 4; i++) px4[i] = (int)rec[13 + i];
  } else if (n_obj > 0) {
    for (int a0 = T; a0 < max_iter; a0 += 64) {  // wave-uniform loop
      const int a = a0 + lane;
      int o = -1, q4[4] = {-1, -1, -1, -1};
      Pose Q;
      const bool acc = a < max_iter && attempt<kDepth>(A, h, a, n_obj, ws, o, q4, Q);
      const uint64_t b = __ballot(acc);
      if (b) {
        const int src = __ffsll((unsigned long long)b) - 1;  // the lowest accepted attempt
        obj = __shfl(o, src);
        for (int i = 0; i < 4; i++) px4[i] = __shfl(q4[i], src);
        for (int i = 0; i < 9; i++) P.R[i] = __shfl(Q.R[i], src);
        for (int i = 0; i < 3; i++) P.t[i] = __shfl(Q.t[i], src);
        break;
      }
    }
  }
  if (lane != 0) return;
  double* hr = ws.hyp + (size_t)h * 16;
  float* ho = hyps_out + (size_t)h * 13;
  hr[0] = obj;
  ho[0] = (float)obj;
  for (int i = 0; i < 12; i++) ho[1 + i] = 0.f;
  for (int i = 0; i < kPx; i++) hyp_px[h * kPx + i] = obj >= 0 ? px4[i] : -1;
  if (obj < 0) {
    hr[0] = -1;
    return;
  }
  for (int i = 0; i < 9; i++) hr[1 + i] = P.R[i];
  for (int i = 0; i < 3; i++) hr[10 + i] = P.t[i];
  for (int i = 0; i < 9; i++) ho[1 + i] = (float)P.R[i];
  for (int i = 0; i < 3; i++) ho[10 + i] = (float)P.t[i];
}

// The preemptive rounds of :1693-1727 as launches over (surviving
// hypothesis, object): per round one workgroup counts one hypothesis's
// inliers over the round's subset (k_p2d_count), then one workgroup per
// object keeps the better half (k_select_sum); survivor lists live in the
// workspace.  k_p2d_collect seeds them (each object's hypotheses in
// ascending h, the stored order -- see the oracle), k_p2d_finish writes the
// output of :1729-1764.
__global__ void __launch_bounds__(64) k_p2d_collect(int n_hyp, P2dWs ws) {  // one wave per object
  const int oi = blockIdx.x, lane = pcnn::lane_id();
  if (oi >= *ws.nobj) return;
  const double obj = ws.objs[oi];
  int m = 0;
  for (int h0 = 0; h0 < n_hyp; h0 += 64) {  // ballot compaction keeps ascending h
    const int h = h0 + lane;
    const bool mine = h < n_hyp && ws.hyp[(size_t)h * 16] == obj;
    const uint64_t b = __ballot(mine);
    if (mine) ws.rl[oi * kMaxHypBlock + m + __popcll(b & pcnn::lanemask_lt())] = h;
    m += __popcll(b);
  }
  if (lane == 0) ws.rm[oi] = m;
}

// grid (hypothesis slot, object, kCntZ): workgroup z counts the subset chunks
// z, z + kCntZ, ... of kCntChunk entries (round 5: one workgroup per
// hypothesis walked the whole subset, 26 us per round) and writes its partial
// count; k_select_sum adds the partials (integers)
__global__ void __launch_bounds__(256) k_p2d_count(const float* __restrict__ vm, const float* __restrict__ ext, int W,
                                                   int C, Cam k, P2dWs ws, int r) {
  __shared__ int part[4];
  const int j = blockIdx.x, oi = blockIdx.y, z = blockIdx.z;
  if (oi >= *ws.nobj || j >= ws.rm[oi]) return;  // block-uniform
  const int obj = ws.objs[oi];
  const int* L = ws.lists + ws.listoff[obj];
  const int h = ws.rl[oi * kMaxHypBlock + j];
  const int* S = ws.sub + (size_t)kRounds * ws.listoff[obj] + (size_t)r * ws.count[obj];
  const int ns = ws.subcnt[obj * kRounds + r];
  const double* hr = ws.hyp + (size_t)h * 16;
  Pose P;
  for (int i = 0; i < 9; i++) P.R[i] = hr[1 + i];
  for (int i = 0; i < 3; i++) P.t[i] = hr[10 + i];
  int cnt = 0;
  for (int c0 = z * kCntChunk; c0 < ns; c0 += (int)gridDim.z * kCntChunk) {  // countInliers2D (:1171-1214)
    for (int i = c0 + threadIdx.x; i < c0 + kCntChunk && i < ns; i += 256) {
      const int idx = L[S[i]];
      const double u0 = idx % W, v0 = idx / W;
      const F3 o = mode3d(vm, ext, C, obj, idx);
      double u, v;
      project(P, D3{o.x, o.y, o.z}, k, u, v);
      if (sqrt((u0 - u) * (u0 - u) + (v0 - v) * (v0 - v)) < 10.0f) cnt++;
    }
  }
  cnt = pcnn::wave_sum(cnt);
  if (pcnn::lane_id() == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) ws.pcnt[((size_t)oi * kMaxHypBlock + j) * kCntZ + z] = part[0] + part[1] + part[2] + part[3];
}

// stable sort by inliers (descending, then list position), keep the better
// half; hl / hc (the m survivors and counts) are in LDS and visible
__device__ void keep_better_half(const P2dWs& ws, int oi, int m, const int* hl, const int* hc, int* tmp) {
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    int rank = 0;
    for (int q = 0; q < m; q++) rank += hc[q] > hc[j] || (hc[q] == hc[j] && q < j);
    tmp[rank] = j;
  }
  __syncthreads();
  const int keep = m / 2;
  for (int j = threadIdx.x; j < keep; j += blockDim.x) {
    ws.rl[oi * kMaxHypBlock + j] = hl[tmp[j]];
    ws.rc[oi * kMaxHypBlock + j] = hc[tmp[j]];
  }
  if (threadIdx.x == 0) ws.rm[oi] = keep;
}

// the round's counts (partials summed: integers) into rc / inl_out, then the
// stable halving (both estimators)
__global__ void __launch_bounds__(1024) k_select_sum(P2dWs ws, int r, int Z, int32_t* __restrict__ inl_out) {
  __shared__ int hl[kMaxHypBlock], hc[kMaxHypBlock], tmp[kMaxHypBlock];
  const int oi = blockIdx.x;
  if (oi >= *ws.nobj) return;
  const int m = ws.rm[oi];
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    const int32_t* pc = ws.pcnt + ((size_t)oi * kMaxHypBlock + j) * kCntZ;
    int c = 0;
    for (int z = 0; z < Z; z++) c += pc[z];
    const int h = ws.rl[oi * kMaxHypBlock + j];
    hl[j] = h;
    hc[j] = c;
    ws.rc[oi * kMaxHypBlock + j] = c;
    inl_out[h * kRounds + r] = c;
  }
  __syncthreads();
  if (m <= 1) return;  // block-uniform
  keep_better_half(ws, oi, m, hl, hc, tmp);
}

__global__ void __launch_bounds__(64) k_p2d_finish(int C, int n_hyp, P2dWs ws, int32_t* __restrict__ final_out,
                                                   float* __restrict__ poses_out) {
  const int oi = blockIdx.x, lane = pcnn::lane_id();  // one wave per object
  if (oi >= *ws.nobj || ws.rm[oi] == 0) return;
  const int obj = ws.objs[oi];
  const int h = ws.rl[oi * kMaxHypBlock];
  int nh = 0;
  for (int q = lane; q < n_hyp; q += 64) nh += ws.hyp[(size_t)q * 16] == (double)obj;
  nh = pcnn::wave_sum(nh);
  if (lane != 0) return;
  final_out[obj * 3] = h;
  final_out[obj * 3 + 1] = ws.rc[oi * kMaxHypBlock];
  final_out[obj * 3 + 2] = nh;
  const double* hr = ws.hyp + (size_t)h * 16;
  for (int y = 0; y < 3; y++)
    for (int x = 0; x < 4; x++) poses_out[obj + C * (y * 4 + x)] = x < 3 ? (float)hr[1 + y * 3 + x] : (float)hr[10 + y];
}

// ===========================================================================
// estimatePose3D (synthesize.cpp:1769-1965) on the device.  The label lists,
// object ids and hypothesis bookkeeping are estimatePose2D's (above); the
// 3-D pieces:
//   k_p3d_eye: getEye / pxToEye (:1372-1407), the camera coordinates of the
//       raw depth (float arithmetic; holes at the origin);
//   k_p3d_valid: one bit per class-list position -- depth present -- so
//       that a round's subset can skip holes the way countInliers3D does
//       (:1255-1287: a hole advances to the next pixel without a draw);
//   k_p3d_subset: the rounds' subsets with holes: positions p_{j+1} =
//       next_valid(p_j + gap_j), the same Philox gaps as estimatePose2D.
//       A class without holes takes the parallel gap scan; otherwise one wave
//       walks 64 draws per step from the class's bits in LDS, the lanes up to
//       the first one landing on a hole accepted at once, that lane moved to
//       the next valid position (a wave-wide bit search) and the walk resumed;
//   k_attempts<true> / k_pick<true>: the sampling loop (:1814-1889);
//   k_p3d_count: countInliers3D over the round's subset (1 cm in double),
//       inlier bits per hypothesis;
//   k_select_sum: the partial counts summed, the stable halving (as
//       estimatePose2D);
//   k_p3d_update: updateHyp3D (:1347-1364) for every survivor, one wave
//       each: filterInliers3D (:1308-1322; pick k of round r on its own
//       stream (draw, h, 'F3D', 1024 r + k)), the inlier ranks resolved to
//       subset positions by a popcount prefix, then the rigid transform with
//       the workgroup-tree sums and the 3x3 Jacobi SVD;
//   k_p3d_finish: the survivor's output (:1936-1964): when it has more than
//       minPixels = 10 inliers, filterInliers3D again (r = 8) and
//       refineWithOpt (:1510-1567) -- the bounded Nelder-Mead over the
//       Rodrigues vector and translation (+-10 deg, +-0.1, +-0.1, +-0.5 m,
//       100 evaluations) of optEnergy3D (:1464-1507), one workgroup per
//       object, the energy's float sum in the workgroup tree.

struct P3dWs {
  P2dWs b;
  float* eye;       // (H W 3) camera coordinates
  uint64_t* valid;  // depth-present bits over the concatenated class lists (+ 2 pad words)
  uint64_t* imask;  // (n_hyp, mwords) inlier bits over the round's subset
  int32_t* pick;    // (n_hyp, kMaxInl) pixels of the last refit's correspondences
  int32_t* npick;   // (n_hyp)
  int mwords;
};

constexpr int kMaxInl = 1000;     // maxPixels: filterInliers3D's cap (:1796)
constexpr int kLdsWords = 5120;   // class-list bits kept in LDS by k_p3d_subset (327,680 positions)
constexpr int kSkipMax = 65536;   // class lists up to this long also get the per-position skip bytes
constexpr int kPrefWords = 2048;  // subset words with an LDS popcount prefix in k_p3d_update
constexpr int kFinThreads = 1024;  // k_p3d_finish workgroup (one correspondence per thread)

// the outputs' initial values (one launch instead of five fills)
__global__ void __launch_bounds__(1024) k_p3d_init(int C, int n_hyp, float* __restrict__ poses_out,
                                                   float* __restrict__ energy_out, int32_t* __restrict__ inl_out,
                                                   int32_t* __restrict__ final_out, int32_t* __restrict__ rm) {
  for (int i = threadIdx.x; i < 12 * C; i += 1024) poses_out[i] = 0.f;
  for (int i = threadIdx.x; i < C; i += 1024) {
    energy_out[i] = 0.f;
    rm[i] = 0;
  }
  for (int i = threadIdx.x; i < 3 * C; i += 1024) final_out[i] = -1;
  for (int i = threadIdx.x; i < kRounds * n_hyp; i += 1024) inl_out[i] = -1;
}

__global__ void __launch_bounds__(256) k_p3d_eye(const uint16_t* __restrict__ depth, int H, int W, float fx, float fy,
                                                 float px, float py, float factor, float* __restrict__ eye) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const int x = p % W, y = p / W;
  const unsigned short d = depth[p];
  float e0 = 0.f, e1 = 0.f, e2 = 0.f;
  if (d != 0) {
    e0 = ((float)x - px) * (float)d / fx / factor;
    e1 = ((float)y - py) * (float)d / fy / factor;
    e2 = (float)d / factor;
  }
  eye[(size_t)p * 3] = e0;
  eye[(size_t)p * 3 + 1] = e1;
  eye[(size_t)p * 3 + 2] = e2;
}

// grid valid_blocks(HW): every word a class_word read may touch is written
inline int valid_blocks(int HW) { return (HW + 64 + 255) / 256; }

__global__ void __launch_bounds__(256) k_p3d_valid(int C, P3dWs w3) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int total = w3.b.listoff[C - 1] + w3.b.count[C - 1];
  const bool v = i < total && w3.eye[(size_t)w3.b.lists[i] * 3 + 2] != 0.f;
  const uint64_t b = __ballot(v);
  if (pcnn::lane_id() == 0) w3.valid[i >> 6] = b;
}

// bits [64 k, 64 k + 64) of the class list starting at global bit o, none past N
__device__ __forceinline__ uint64_t class_word(const uint64_t* __restrict__ V, long o, int N, long k) {
  const long b = o + 64 * k;
  const long w = b >> 6;
  const int sh = (int)(b & 63);
  uint64_t v = V[w] >> sh;
  if (sh) v |= V[w + 1] << (64 - sh);
  const long rem = (long)N - 64 * k;
  if (rem < 64) v &= rem <= 0 ? 0ull : ((1ull << rem) - 1);
  return v;
}

__global__ void __launch_bounds__(1024) k_p3d_subset(uint64_t seed, P3dWs w3) {
  __shared__ uint64_t bits[kLdsWords];  // 40 KiB
  __shared__ uint8_t skip[kSkipMax];     // 64 KiB
  __shared__ int wsum[16];
  __shared__ long qrel[1024];
  __shared__ int sh_int[4];
  const P2dWs& ws = w3.b;
  const int c = blockIdx.x, r = blockIdx.y, t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
  const int N = ws.count[c];
  if (c == 0 || !((float)N > 400.0f)) return;  // not an object (block-uniform)
  int* S = ws.sub + (size_t)kRounds * ws.listoff[c] + (size_t)r * N;
  int* cnt_out = ws.subcnt + c * kRounds + r;
  const long o = ws.listoff[c];
  const int nw = (N + 63) / 64;
  const bool in_lds = nw <= kLdsWords;
  int nv = 0;
  for (int k = t; k < nw; k += 1024) {
    const uint64_t v = class_word(w3.valid, o, N, k);
    if (in_lds) bits[k] = v;
    nv += __popcll(v);
  }
  nv = pcnn::wave_sum(nv);
  if (t == 0) sh_int[0] = 0;
  __syncthreads();
  if (lane == 0) atomicAdd(&sh_int[0], nv);  // integer: order-free
  __syncthreads();
  nv = sh_int[0];
  auto word = [&](long k) -> uint64_t { return in_lds ? bits[k] : class_word(w3.valid, o, N, k); };
  const int maxPixels = 1000 * (r + 1);
  const float rate = maxPixels / (float)N;  // :1250
  if (!(rate < 1)) {  // every valid pixel in list order (:1283-1286)
    long carry = 0;
    for (int base = 0; base < nw; base += 1024) {  // ordered compaction, a word per thread
      const int k = base + t;
      const uint64_t v = k < nw ? word(k) : 0ull;
      const int pc = __popcll(v);
      int incl = pc;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      if (lane == 63) wsum[wave] = incl;
      __syncthreads();
      long wb = 0, tot = 0;
      for (int w = 0; w < 16; w++) {
        if (w < wave) wb += wsum[w];
        tot += wsum[w];
      }
      long pos = carry + wb + incl - pc;
      for (uint64_t m = v; m; m &= m - 1) S[pos++] = 64 * k + __ffsll((unsigned long long)m) - 1;
      __syncthreads();
      carry += tot;
    }
    if (t == 0) *cnt_out = nv;
    return;
  }
  const double q = 1.0 - (double)rate;
  if (nv == N) {  // no holes: estimatePose2D's subset
    subset_nohole(seed, c, r, N, q, S, cnt_out, wsum);
    return;
  }
  // skip[x] = next_valid(x) - x (0: x valid; 255: 255 or more, resolved by a
  // word search) when the class list fits kSkipMax bytes: one LDS byte per
  // walk step decides both "hole?" and "how far"
  const bool use_skip = N <= kSkipMax;  // block-uniform
  if (use_skip) {
    for (int x = t; x < N; x += 1024) {
      const int k = x >> 6;
      uint64_t w = word(k) >> (x & 63);
      int d = 0;
      if (!(w & 1ull)) {
        if (w) {
          d = __ffsll((unsigned long long)w) - 1;
        } else {
          d = 64 - (x & 63);
          for (int kk = k + 1; d < 255; kk++, d += 64) {
            if (kk >= nw) {
              d = N - x;  // no valid position after x: the walk leaves the list
              break;
            }
            const uint64_t v = word(kk);
            if (v) {
              d += __ffsll((unsigned long long)v) - 1;
              break;
            }
          }
        }
      }
      skip[x] = (uint8_t)(d < 255 ? d : 255);
    }
    __syncthreads();
  }
  long carry = 0;  // q_{j0}: the hole-free position of draw j0
  long D = 0;      // holes skipped so far (wave 0)
  for (int j0 = 0;; j0 += 1024) {
    const int g = p2d_gap(seed, c, r, j0 + t, q);
    int incl = g;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    long wb = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
      if (w < wave) wb += wsum[w];
      tot += wsum[w];
    }
    qrel[t] = wb + incl - g;
    __syncthreads();
    if (wave == 0 && use_skip) {  // the lean walk: 32-bit positions, one LDS byte per step
      int done = 0, cnt = 0, Di = (int)D;  // D < N <= kSkipMax
      for (int sc = 0; sc < 16 && !done; sc++) {
        const int jl = sc * 64 + lane;
        const long ql = carry + qrel[jl];
        const int qj = ql < N ? (int)ql : N;  // every position at or past N means "past the list"
        int s = 0, pos = 0, nvalid = 64;
        for (;;) {  // wave-uniform; one hole hit resolved per step
          const int x = qj + Di;
          const int hv = x < N ? (int)skip[x] : 0;
          const bool ev = lane >= s && (x >= N || hv != 0);
          const uint64_t b = __ballot(ev);
          const int first = b ? __ffsll((unsigned long long)b) - 1 : 64;
          if (lane >= s && lane < first) pos = x;
          if (first == 64) break;
          const int xs = __builtin_amdgcn_readlane(x, first);
          int hs = __builtin_amdgcn_readlane(hv, first);
          if (xs < N && hs == 255) {  // a run of 255 or more holes: the word search
            long nh = N;
            for (long kb = (xs >> 6); kb < nw; kb += 64) {
              const long k = kb + lane;
              uint64_t v = k < nw ? bits[k] : 0ull;
              if (k == (xs >> 6)) v &= ~0ull << (xs & 63);
              const uint64_t hit = __ballot(v != 0ull);
              if (hit) {
                const int l = __ffsll((unsigned long long)hit) - 1;
                const uint64_t vv = __shfl((unsigned long long)v, l, 64);
                nh = 64 * (kb + l) + __ffsll((unsigned long long)vv) - 1;
                break;
              }
            }
            hs = (int)(nh - xs);
          }
          if (xs >= N || xs + hs >= N) {  // the walk leaves the list
            done = 1;
            cnt = j0 + sc * 64 + first;
            nvalid = first;
            break;
          }
          Di += hs;
          s = first;
        }
        if (lane < nvalid) S[j0 + jl] = pos;
      }
      D = Di;
      if (lane == 0) {
        sh_int[1] = done;
        sh_int[2] = cnt;
      }
    } else if (wave == 0) {  // class lists longer than kSkipMax: the bit walk
      int done = 0, cnt = 0;
      for (int sc = 0; sc < 16 && !done; sc++) {
        const int jl = sc * 64 + lane;
        const long qj = carry + qrel[jl];
        int s = 0;
        for (;;) {  // wave-uniform; one hole hit resolved per step
          const long x = qj + D;
          bool ev = false;
          if (lane >= s) ev = x >= N || !((word(x >> 6) >> (x & 63)) & 1ull);
          const uint64_t b = __ballot(ev);
          const int first = b ? __ffsll((unsigned long long)b) - 1 : 64;
          if (lane >= s && lane < first) S[j0 + jl] = (int)x;
          if (first == 64) break;
          const long xs = __shfl(x, first, 64);
          long nh = N;
          const uint64_t w0 = xs < N ? word(xs >> 6) >> (xs & 63) : 0ull;
          if (w0) {  // the hole run ends in this word (the usual case)
            nh = xs + __ffsll((unsigned long long)w0) - 1;
          } else if (xs < N) {  // the next valid position past this word (wave-wide word search)
            for (long kb = (xs >> 6) + 1; kb < nw; kb += 64) {
              const long k = kb + lane;
              const uint64_t v = k < nw ? word(k) : 0ull;
              const uint64_t hit = __ballot(v != 0ull);
              if (hit) {
                const int l = __ffsll((unsigned long long)hit) - 1;
                const uint64_t vv = __shfl((unsigned long long)v, l, 64);
                nh = 64 * (kb + l) + __ffsll((unsigned long long)vv) - 1;
                break;
              }
            }
          }
          if (nh >= N) {  // the walk leaves the list: draws j0 + sc 64 + first .. are not taken
            done = 1;
            cnt = j0 + sc * 64 + first;
            break;
          }
          D += nh - xs;
          s = first;
        }
      }
      if (lane == 0) {
        sh_int[1] = done;
        sh_int[2] = cnt;
      }
    }
    __syncthreads();
    if (sh_int[1]) {
      if (t == 0) *cnt_out = sh_int[2];
      return;
    }
    carry += tot;
  }
}

// grid (hypothesis slot, object, kCntZ): workgroup z takes the subset chunks
// z, z + kCntZ, ... of kCntChunk entries and writes its partial count (the
// chunks' inlier bits go to the hypothesis's mask)
__global__ void __launch_bounds__(256) k_p3d_count(const float* __restrict__ vm, const float* __restrict__ ext, int C,
                                                   P3dWs w3, int r) {
  __shared__ int part[4];
  const P2dWs& ws = w3.b;
  const int j = blockIdx.x, oi = blockIdx.y, z = blockIdx.z, lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  if (oi >= *ws.nobj || j >= ws.rm[oi]) return;  // block-uniform
  const int obj = ws.objs[oi];
  const int* L = ws.lists + ws.listoff[obj];
  const int h = ws.rl[oi * kMaxHypBlock + j];
  const int* S = ws.sub + (size_t)kRounds * ws.listoff[obj] + (size_t)r * ws.count[obj];
  const int ns = ws.subcnt[obj * kRounds + r];
  const double* hr = ws.hyp + (size_t)h * 16;
  Pose P;
  for (int i = 0; i < 9; i++) P.R[i] = hr[1 + i];
  for (int i = 0; i < 3; i++) P.t[i] = hr[10 + i];
  uint64_t* M = w3.imask + (size_t)h * w3.mwords;
  int cnt = 0;
  for (int c0 = z * kCntChunk; c0 < ns; c0 += (int)gridDim.z * kCntChunk) {  // countInliers3D (:1255-1287)
    for (int i0 = c0; i0 < c0 + kCntChunk && i0 < ns; i0 += 256) {
      const int i = i0 + threadIdx.x;
      bool in = false;
      if (i < ns) {
        const int p = L[S[i]];
        const F3 e = eye_at(w3.eye, p);
        const F3 o = mode3d(vm, ext, C, obj, p);
        in = nrm(sub(D3{e.x, e.y, e.z}, xform(P, D3{o.x, o.y, o.z}))) < 0.01;
      }
      const uint64_t b = __ballot(in);
      if (lane == 0 && i0 + 64 * wave < ns) M[(i0 >> 6) + wave] = b;
      cnt += in;
    }
  }
  cnt = pcnn::wave_sum(cnt);
  if (lane == 0) part[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) ws.pcnt[((size_t)oi * kMaxHypBlock + j) * kCntZ + z] = part[0] + part[1] + part[2] + part[3];
}

// the subset position of the rank-th set bit of M (pref: exclusive popcount
// prefix per word when the subset has at most kPrefWords words)
__device__ __forceinline__ int select_bit(const uint64_t* __restrict__ M, const int* pref, int nw, int rank) {
  int k = 0;
  if (nw <= kPrefWords) {
    int lo = 0, hi = nw - 1;  // the last word with pref <= rank
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pref[mid] <= rank) lo = mid; else hi = mid - 1;
    }
    k = lo;
    rank -= pref[k];
  } else {
    for (;; k++) {
      const int pc = __popcll(M[k]);
      if (rank < pc) break;
      rank -= pc;
    }
  }
  uint64_t v = M[k];  // the rank-th set bit of v by halving
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = (1ull << w) - 1;
    const int c = __popcll(v & low);
    if (rank >= c) {
      rank -= c;
      v >>= w;
      pos += w;
    } else {
      v &= low;
    }
  }
  return 64 * k + pos;
}

// one workgroup per survivor: the popcount prefix and the picks spread over
// 1024 threads (each pick on its own stream, one correspondence per thread),
// the centroid and covariance sums in the workgroup tree, the SVD on thread 0
__global__ void __launch_bounds__(1024) k_p3d_update(const float* __restrict__ vm, const float* __restrict__ ext,
                                                     int C, uint64_t seed, P3dWs w3, int r) {
  __shared__ int pref[kPrefWords];
  __shared__ int wsum[16];
  __shared__ double wc[16][6], wv[16][9];
  const P2dWs& ws = w3.b;
  const int j = blockIdx.x, oi = blockIdx.y, t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
  if (oi >= *ws.nobj || j >= ws.rm[oi]) return;  // block-uniform
  const int n = ws.rc[oi * kMaxHypBlock + j];
  if (n < 4) return;  // :1350-1351
  const int obj = ws.objs[oi];
  const int h = ws.rl[oi * kMaxHypBlock + j];
  const int* L = ws.lists + ws.listoff[obj];
  const int* S = ws.sub + (size_t)kRounds * ws.listoff[obj] + (size_t)r * ws.count[obj];
  const int ns = ws.subcnt[obj * kRounds + r];
  const int nw = (ns + 63) / 64;
  const uint64_t* M = w3.imask + (size_t)h * w3.mwords;
  if (nw <= kPrefWords) {  // block-uniform
    int carry = 0;
    for (int base = 0; base < nw; base += 1024) {
      const int k = base + t;
      const int pc = k < nw ? __popcll(M[k]) : 0;
      int incl = pc;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      if (lane == 63) wsum[wave] = incl;
      __syncthreads();
      int wb = 0, tot = 0;
      for (int w = 0; w < 16; w++) {
        if (w < wave) wb += wsum[w];
        tot += wsum[w];
      }
      if (k < nw) pref[k] = carry + wb + incl - pc;
      __syncthreads();
      carry += tot;
    }
  }
  const int m = n >= kMaxInl ? kMaxInl : n;  // filterInliers3D (:1308-1322)
  const bool live = t < m;
  double a[3] = {0.0, 0.0, 0.0}, b[3] = {0.0, 0.0, 0.0};
  if (live) {
    int rank = t;
    if (n >= kMaxInl) {
      Stream rs(seed, (uint32_t)h, kTagF3D, (uint32_t)(1024 * r + t));
      rank = rs.uniform(n);
    }
    const int p = L[S[select_bit(M, pref, nw, rank)]];
    const F3 o = mode3d(vm, ext, C, obj, p);
    const F3 e = eye_at(w3.eye, p);
    a[0] = o.x; a[1] = o.y; a[2] = o.z;
    b[0] = e.x; b[1] = e.y; b[2] = e.z;
    w3.pick[(size_t)h * kMaxInl + t] = p;
  }
  if (t == 0) w3.npick[h] = m;
  // Hypothesis::refine (:1359): calcRigidBodyTransform's sums in the tree
  for (int i = 0; i < 3; i++) {
    const double sa = wave_fold(live ? 0.0 + a[i] : 0.0), sb = wave_fold(live ? 0.0 + b[i] : 0.0);
    if (lane == 0) {
      wc[wave][i] = sa;
      wc[wave][3 + i] = sb;
    }
  }
  __syncthreads();
  const double inv = 1.0 / (double)m;
  double cA[3], cB[3];
  for (int i = 0; i < 3; i++) {
    cA[i] = cross_fold<double, 6>(wc, i) * inv;
    cB[i] = cross_fold<double, 6>(wc, 3 + i) * inv;
  }
  for (int rr = 0; rr < 3; rr++)
    for (int cc = 0; cc < 3; cc++) {
      const double v = wave_fold(live ? 0.0 + (a[rr] - cA[rr]) * (b[cc] - cB[cc]) : 0.0);
      if (lane == 0) wv[wave][rr * 3 + cc] = v;
    }
  __syncthreads();
  if (t != 0) return;
  double Hc[9];
  for (int i = 0; i < 9; i++) Hc[i] = cross_fold<double, 9>(wv, i);
  const Pose P = rigid_from_cov_ool(Hc, cA, cB);
  double* hr = ws.hyp + (size_t)h * 16;
  for (int i = 0; i < 9; i++) hr[1 + i] = P.R[i];
  for (int i = 0; i < 3; i++) hr[10 + i] = P.t[i];
}

// one workgroup per object: the final filter, then refineWithOpt as the
// bounded Nelder-Mead of k_nm (icp.hip): thread 0 keeps the simplex in LDS,
// each thread holds one correspondence, and every evaluation sums the
// distances in the workgroup tree (the oracle's order)
__global__ void __launch_bounds__(kFinThreads) k_p3d_finish(const float* __restrict__ vm,
                                                            const float* __restrict__ ext, int C, int n_hyp,
                                                            uint64_t seed, int nm_evals, P3dWs w3,
                                                            int32_t* __restrict__ final_out,
                                                            float* __restrict__ poses_out,
                                                            float* __restrict__ energy_out) {
  constexpr int nd = 6;
  __shared__ float wf[16][1];
  __shared__ double pts[nd + 1][nd], vals[nd + 1], lb[nd], ub[nd], xq[nd], xr[nd], cen[nd];
  __shared__ float Rf[9];
  __shared__ int nh_s;
  const P2dWs& ws = w3.b;
  const int oi = blockIdx.x, t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
  if (oi >= *ws.nobj || ws.rm[oi] == 0) return;  // block-uniform
  const int obj = ws.objs[oi];
  const int h = ws.rl[oi * kMaxHypBlock];
  const int n = ws.rc[oi * kMaxHypBlock];
  if (t == 0) nh_s = 0;
  __syncthreads();
  {
    int nh = 0;
    for (int q = t; q < n_hyp; q += kFinThreads) nh += ws.hyp[(size_t)q * 16] == (double)obj;
    nh = pcnn::wave_sum(nh);
    if (lane == 0) atomicAdd(&nh_s, nh);  // integer: order-free
  }
  const double* hr = ws.hyp + (size_t)h * 16;
  Pose P;
  for (int i = 0; i < 9; i++) P.R[i] = hr[1 + i];
  for (int i = 0; i < 3; i++) P.t[i] = hr[10 + i];
  float en = 0.f;
  if (n > 10) {  // minPixels (:1939); block-uniform
    const int mp = w3.npick[h];
    const int m = mp >= kMaxInl ? kMaxInl : mp;
    float co[3] = {0.f, 0.f, 0.f}, ce[3] = {0.f, 0.f, 0.f};
    const bool live = t < m;
    if (live) {  // filterInliers3D again (:1942): correspondence t of this thread
      int idx = t;
      if (mp >= kMaxInl) {
        Stream rs(seed, (uint32_t)h, kTagF3D, (uint32_t)(1024 * kRounds + t));
        idx = rs.uniform(mp);
      }
      const int p = w3.pick[(size_t)h * kMaxInl + idx];
      const F3 o = mode3d(vm, ext, C, obj, p);
      const F3 e = eye_at(w3.eye, p);
      co[0] = o.x; co[1] = o.y; co[2] = o.z;
      ce[0] = e.x; ce[1] = e.y; ce[2] = e.z;
    }
    auto eval = [&]() -> double {  // optEnergy3D (:1464-1507) at xq (written by thread 0)
      if (t == 0) {
        double Rd[9];
        rod_v2m(xq, Rd);
        for (int i = 0; i < 9; i++) Rf[i] = (float)Rd[i];  // jp::double2float
      }
      __syncthreads();
      float leaf = 0.f;
      if (live) {
        float tr[3];
        for (int rr = 0; rr < 3; rr++) {
          const float mm = Rf[rr * 3 + 0] * co[0] + Rf[rr * 3 + 1] * co[1] + Rf[rr * 3 + 2] * co[2];
          tr[rr] = (float)((double)mm + xq[3 + rr]);
        }
        const double dx = (double)tr[0] - (double)ce[0], dy = (double)tr[1] - (double)ce[1],
                     dz = (double)tr[2] - (double)ce[2];
        leaf = 0.f + (float)sqrt(dx * dx + dy * dy + dz * dz);
      }
      const float sw = wave_fold(leaf);
      if (lane == 0) wf[wave][0] = sw;
      __syncthreads();
      // every thread folds the 16 wave sums (the next evaluation's first
      // barrier orders these reads before wf is rewritten)
      return (double)(cross_fold<float, 1>(wf, 0) / (float)m);
    };
    auto clampq = [&](int e, double v) { return fmin(fmax(v, lb[e]), ub[e]); };
    if (t == 0) {  // refineWithOpt (:1510-1567)
      double x0[nd];
      rod_m2v(P.R, x0);
      for (int i = 0; i < 3; i++) x0[3 + i] = P.t[i];
      const double rot = 10 * 3.1415926 / 180;  // rotRange, PI of types.h:33
      const double rng[nd] = {rot, rot, rot, 0.1, 0.1, 0.5};
      for (int i = 0; i < nd; i++) {
        lb[i] = x0[i] - rng[i];
        ub[i] = x0[i] + rng[i];
        pts[0][i] = x0[i];
      }
      for (int i = 0; i < nd; i++) {
        const double st = fmin(0.25 * (ub[i] - lb[i]), fmin(0.75 * (ub[i] - x0[i]), 0.75 * (x0[i] - lb[i])));
        for (int e = 0; e < nd; e++) pts[i + 1][e] = e == i ? x0[e] + st : x0[e] + 0.0;
      }
    }
    for (int i = 0; i <= nd; i++) {
      if (t == 0)
        for (int e = 0; e < nd; e++) xq[e] = pts[i][e];
      const double v = eval();
      if (t == 0) vals[i] = v;
    }
    int nev = nd + 1;
    while (nev < nm_evals) {  // nev is identical in every thread
      if (t == 0) {
        for (int i = 1; i <= nd; i++)
          for (int jj = i; jj > 0 && vals[jj] < vals[jj - 1]; jj--) {
            const double tv = vals[jj];
            vals[jj] = vals[jj - 1];
            vals[jj - 1] = tv;
            for (int e = 0; e < nd; e++) {
              const double tp = pts[jj][e];
              pts[jj][e] = pts[jj - 1][e];
              pts[jj - 1][e] = tp;
            }
          }
        for (int e = 0; e < nd; e++) {
          double sm = pts[0][e];
          for (int i = 1; i < nd; i++) sm = sm + pts[i][e];
          cen[e] = sm / (double)nd;
        }
        for (int e = 0; e < nd; e++) {
          xr[e] = clampq(e, cen[e] + (cen[e] - pts[nd][e]));
          xq[e] = xr[e];
        }
      }
      const double fr = eval();
      nev++;
      const double v0 = vals[0], vn1 = vals[nd - 1], vn = vals[nd];
      if (fr < v0 && nev < nm_evals) {
        if (t == 0)
          for (int e = 0; e < nd; e++) xq[e] = clampq(e, cen[e] + 2.0 * (cen[e] - pts[nd][e]));
        const double fe = eval();
        nev++;
        if (t == 0) {
          const bool ex = fe < fr;
          for (int e = 0; e < nd; e++) pts[nd][e] = ex ? xq[e] : xr[e];
          vals[nd] = ex ? fe : fr;
        }
      } else if (fr < vn1) {
        if (t == 0) {
          for (int e = 0; e < nd; e++) pts[nd][e] = xr[e];
          vals[nd] = fr;
        }
      } else if (nev < nm_evals) {
        if (t == 0)
          for (int e = 0; e < nd; e++)
            xq[e] = fr >= vn ? clampq(e, cen[e] + 0.5 * (pts[nd][e] - cen[e])) : clampq(e, cen[e] + 0.5 * (xr[e] - cen[e]));
        const double fc = eval();
        nev++;
        if (fc < fmin(fr, vn)) {
          if (t == 0) {
            for (int e = 0; e < nd; e++) pts[nd][e] = xq[e];
            vals[nd] = fc;
          }
        } else {
          const int sm = min(nd, nm_evals - nev);
          for (int i = 1; i <= sm; i++) {  // shrink toward the best
            if (t == 0)
              for (int e = 0; e < nd; e++) xq[e] = clampq(e, pts[0][e] + 0.5 * (pts[i][e] - pts[0][e]));
            const double fv = eval();
            if (t == 0) {
              for (int e = 0; e < nd; e++) pts[i][e] = xq[e];
              vals[i] = fv;
            }
          }
          nev += sm > 0 ? sm : 0;
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      int bi = 0;
      for (int i = 1; i <= nd; i++)
        if (vals[i] < vals[bi]) bi = i;
      double xb[nd];
      for (int e = 0; e < nd; e++) xb[e] = pts[bi][e];
      rod_v2m(xb, P.R);
      for (int i = 0; i < 3; i++) P.t[i] = xb[3 + i];
      en = (float)vals[bi];
    }
  }
  __syncthreads();
  if (t != 0) return;
  final_out[obj * 3] = h;
  final_out[obj * 3 + 1] = n;
  final_out[obj * 3 + 2] = nh_s;
  energy_out[obj] = en;
  for (int y = 0; y < 3; y++)
    for (int x = 0; x < 4; x++) poses_out[obj + C * (y * 4 + x)] = x < 3 ? (float)P.R[y * 3 + x] : (float)P.t[y];
}

struct Layout {
  size_t colcnt, coloff, count, lists, listoff, objs, nobj, subcnt, hyp, att, rl, rc, rm, pcnt, sub, total;
};

Layout layout(int H, int W, int C, int n_hyp) {
  // byte offsets of the regions (256-B aligned) inside the caller's workspace
  size_t off = 0;
  auto take = [&](size_t bytes) {
    off = pcnn::align_up(off, 256);
    const size_t o = off;
    off += bytes;
    return o;
  };
  Layout l;
  l.colcnt = take((size_t)C * W * sizeof(int32_t));
  l.coloff = take((size_t)C * W * sizeof(int32_t));
  l.count = take((size_t)C * sizeof(int32_t));
  l.lists = take((size_t)H * W * sizeof(int32_t));
  l.listoff = take((size_t)C * sizeof(int32_t));
  l.objs = take((size_t)C * sizeof(int32_t));
  l.nobj = take(sizeof(int32_t));
  l.subcnt = take((size_t)C * kRounds * sizeof(int32_t));
  l.hyp = take((size_t)n_hyp * 16 * sizeof(double));
  l.att = take((size_t)n_hyp * kAttempts * kAttRec * sizeof(double));
  l.rl = take((size_t)C * kMaxHypBlock * sizeof(int32_t));
  l.rc = take((size_t)C * kMaxHypBlock * sizeof(int32_t));
  l.rm = take((size_t)C * sizeof(int32_t));
  l.pcnt = take((size_t)C * kMaxHypBlock * kCntZ * sizeof(int32_t));
  // subsets: a round visits at most every pixel of the class once
  l.sub = take((size_t)kRounds * H * W * sizeof(int32_t));
  l.total = off + 256;
  return l;
}

}  // namespace

extern "C" size_t pcnn_pose2d_workspace_size(int H, int W, int C, int n_hyp) {
  if (H <= 0 || W <= 0 || C <= 0 || n_hyp <= 0) return 256;
  return layout(H, W, C, n_hyp).total;
}

extern "C" int pcnn_pose2d(const int32_t* label, const float* vertmap, const float* extents, int H, int W, int C,
                           float fx, float fy, float px, float py, uint64_t seed, int n_hyp, int max_iter,
                           float* poses_out, float* hyps_out, int32_t* hyp_px, int32_t* inl_out, int32_t* final_out,
                           void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(label && vertmap && extents && poses_out && hyps_out && hyp_px && inl_out && final_out);
  // n_hyp <= 256: the reference's ransacIterations (:1601), so that 8 halving
  // rounds leave one hypothesis per object, as getWorkingQueue (:1150-1160)
  // stops at
  PCNN_REQUIRE(H > 0 && W > 0 && C > 1 && C <= 64 && n_hyp > 0 && n_hyp <= kMaxHyp && max_iter > 0);
  PCNN_REQUIRE((long)H * W < (1l << 28));
  const Layout l = layout(H, W, C, n_hyp);
  if (!workspace || workspace_bytes < l.total) return PCNN_ECAPACITY;
  char* base = (char*)workspace;
  P2dWs ws;
  ws.colcnt = (int32_t*)(base + l.colcnt);
  ws.coloff = (int32_t*)(base + l.coloff);
  ws.count = (int32_t*)(base + l.count);
  ws.lists = (int32_t*)(base + l.lists);
  ws.listoff = (int32_t*)(base + l.listoff);
  ws.objs = (int32_t*)(base + l.objs);
  ws.nobj = (int32_t*)(base + l.nobj);
  ws.subcnt = (int32_t*)(base + l.subcnt);
  ws.hyp = (double*)(base + l.hyp);
  ws.att = (double*)(base + l.att);
  ws.rl = (int32_t*)(base + l.rl);
  ws.rc = (int32_t*)(base + l.rc);
  ws.rm = (int32_t*)(base + l.rm);
  ws.pcnt = (int32_t*)(base + l.pcnt);
  ws.sub = (int32_t*)(base + l.sub);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(poses_out, 0, (size_t)12 * C * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
  if (hipMemsetAsync(inl_out, 0xFF, (size_t)n_hyp * kRounds * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  if (hipMemsetAsync(final_out, 0xFF, (size_t)C * 3 * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  if (hipMemsetAsync(ws.rm, 0, (size_t)C * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  const Cam k{fx, fy, px, py};
  // every count, object list and subset stays on the device: the call is
  // asynchronous on `stream` (round 5; it used to read the class counts
  // back and draw the subsets on host threads)
  hipLaunchKernelGGL(k_p2d_colcount, dim3((W + 3) / 4), dim3(256), 0, st, label, H, W, C, ws.colcnt);
  hipLaunchKernelGGL(k_p2d_scan, dim3(C), dim3(1024), 0, st, ws.colcnt, W, ws.coloff, ws.count);
  hipLaunchKernelGGL(k_p2d_objs, dim3(1), dim3(64), 0, st, C, ws);
  hipLaunchKernelGGL(k_p2d_scatter, dim3((W + 3) / 4), dim3(256), 0, st, label, H, W, C, ws);
  hipLaunchKernelGGL(k_p2d_subset, dim3(C, kRounds), dim3(1024), 0, st, seed, ws);
  const int T = max_iter < kAttempts ? max_iter : kAttempts;
  const AttArgs A{vertmap, extents, nullptr, H, W, C, k, seed};
  hipLaunchKernelGGL(k_attempts<false>, dim3((n_hyp * T + 63) / 64), dim3(64), 0, st, A, n_hyp, T, ws);
  hipLaunchKernelGGL(k_pick<false>, dim3(n_hyp), dim3(64), 0, st, A, n_hyp, max_iter, T, ws, hyps_out, hyp_px);
  hipLaunchKernelGGL(k_p2d_collect, dim3(C), dim3(64), 0, st, n_hyp, ws);
  for (int r = 0; r < kRounds; r++) {
    const int gx = std::max(1, n_hyp >> r);  // survivors halve each round (one stays one)
    hipLaunchKernelGGL(k_p2d_count, dim3(gx, C, count_z(r)), dim3(256), 0, st, vertmap, extents, W, C, k, ws, r);
    hipLaunchKernelGGL(k_select_sum, dim3(C), dim3(1024), 0, st, ws, r, count_z(r), inl_out);
  }
  hipLaunchKernelGGL(k_p2d_finish, dim3(C), dim3(64), 0, st, C, n_hyp, ws, final_out, poses_out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

namespace {

struct Layout3 {
  Layout b;
  size_t eye, valid, imask, pick, npick, total;
  int mwords;
};

Layout3 layout3(int H, int W, int C, int n_hyp) {
  Layout3 l;
  l.b = layout(H, W, C, n_hyp);
  size_t off = l.b.total;
  auto take = [&](size_t bytes) {
    off = pcnn::align_up(off, 256);
    const size_t o = off;
    off += bytes;
    return o;
  };
  const long HW = (long)H * W;
  l.mwords = (int)((HW + 63) / 64);
  l.eye = take((size_t)HW * 3 * sizeof(float));
  l.valid = take((size_t)valid_blocks((int)HW) * 4 * sizeof(uint64_t));
  l.imask = take((size_t)n_hyp * l.mwords * sizeof(uint64_t));
  l.pick = take((size_t)n_hyp * kMaxInl * sizeof(int32_t));
  l.npick = take((size_t)n_hyp * sizeof(int32_t));
  l.total = off + 256;
  return l;
}

P2dWs carve2(char* base, const Layout& l) {
  P2dWs ws;
  ws.colcnt = (int32_t*)(base + l.colcnt);
  ws.coloff = (int32_t*)(base + l.coloff);
  ws.count = (int32_t*)(base + l.count);
  ws.lists = (int32_t*)(base + l.lists);
  ws.listoff = (int32_t*)(base + l.listoff);
  ws.objs = (int32_t*)(base + l.objs);
  ws.nobj = (int32_t*)(base + l.nobj);
  ws.subcnt = (int32_t*)(base + l.subcnt);
  ws.hyp = (double*)(base + l.hyp);
  ws.att = (double*)(base + l.att);
  ws.rl = (int32_t*)(base + l.rl);
  ws.rc = (int32_t*)(base + l.rc);
  ws.rm = (int32_t*)(base + l.rm);
  ws.pcnt = (int32_t*)(base + l.pcnt);
  ws.sub = (int32_t*)(base + l.sub);
  return ws;
}

}  // namespace

extern "C" size_t pcnn_pose3d_workspace_size(int H, int W, int C, int n_hyp) {
  if (H <= 0 || W <= 0 || C <= 0 || n_hyp <= 0) return 256;
  return layout3(H, W, C, n_hyp).total;
}

extern "C" int pcnn_pose3d(const int32_t* label, const uint16_t* depth, const float* vertmap, const float* extents,
                           int H, int W, int C, float fx, float fy, float px, float py, float depth_factor,
                           uint64_t seed, int n_hyp, int max_iter, int nm_evals, float* poses_out, float* hyps_out,
                           int32_t* hyp_px, int32_t* inl_out, int32_t* final_out, float* energy_out, float* eye_out,
                           void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(label && depth && vertmap && extents && poses_out && hyps_out && hyp_px && inl_out && final_out &&
               energy_out);
  // nm_evals >= 7: at least the six-dimensional search's initial simplex (NLopt's
  // maxeval counts it; a smaller budget is refused rather than overrun)
  PCNN_REQUIRE(H > 0 && W > 0 && C > 1 && C <= 64 && n_hyp > 0 && n_hyp <= kMaxHyp && max_iter > 0 && nm_evals >= 7);
  PCNN_REQUIRE((long)H * W < (1l << 28));
  const Layout3 l = layout3(H, W, C, n_hyp);
  if (!workspace || workspace_bytes < l.total) return PCNN_ECAPACITY;
  char* base = (char*)workspace;
  P3dWs w3;
  w3.b = carve2(base, l.b);
  w3.eye = (float*)(base + l.eye);
  w3.valid = (uint64_t*)(base + l.valid);
  w3.imask = (uint64_t*)(base + l.imask);
  w3.pick = (int32_t*)(base + l.pick);
  w3.npick = (int32_t*)(base + l.npick);
  w3.mwords = l.mwords;
  const P2dWs& ws = w3.b;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_p3d_init, dim3(1), dim3(1024), 0, st, C, n_hyp, poses_out, energy_out, inl_out, final_out,
                     ws.rm);
  const Cam k{fx, fy, px, py};
  const int HW = H * W;
  hipLaunchKernelGGL(k_p3d_eye, dim3((HW + 255) / 256), dim3(256), 0, st, depth, H, W, fx, fy, px, py, depth_factor,
                     w3.eye);
  hipLaunchKernelGGL(k_p2d_colcount, dim3((W + 3) / 4), dim3(256), 0, st, label, H, W, C, ws.colcnt);
  hipLaunchKernelGGL(k_p2d_scan, dim3(C), dim3(1024), 0, st, ws.colcnt, W, ws.coloff, ws.count);
  hipLaunchKernelGGL(k_p2d_objs, dim3(1), dim3(64), 0, st, C, ws);
  hipLaunchKernelGGL(k_p2d_scatter, dim3((W + 3) / 4), dim3(256), 0, st, label, H, W, C, ws);
  hipLaunchKernelGGL(k_p3d_valid, dim3(valid_blocks(HW)), dim3(256), 0, st, C, w3);
  hipLaunchKernelGGL(k_p3d_subset, dim3(C, kRounds), dim3(1024), 0, st, seed, w3);
  const int T = max_iter < kAttempts ? max_iter : kAttempts;
  const AttArgs A{vertmap, extents, w3.eye, H, W, C, k, seed};
  hipLaunchKernelGGL(k_attempts<true>, dim3((n_hyp * T + 63) / 64), dim3(64), 0, st, A, n_hyp, T, ws);
  hipLaunchKernelGGL(k_pick<true>, dim3(n_hyp), dim3(64), 0, st, A, n_hyp, max_iter, T, ws, hyps_out, hyp_px);
  hipLaunchKernelGGL(k_p2d_collect, dim3(C), dim3(64), 0, st, n_hyp, ws);
  for (int r = 0; r < kRounds; r++) {
    const int gx = std::max(1, n_hyp >> r);  // survivors halve each round (one stays one)
    hipLaunchKernelGGL(k_p3d_count, dim3(gx, C, count_z(r)), dim3(256), 0, st, vertmap, extents, C, w3, r);
    hipLaunchKernelGGL(k_select_sum, dim3(C), dim3(1024), 0, st, ws, r, count_z(r), inl_out);
    hipLaunchKernelGGL(k_p3d_update, dim3(std::max(1, n_hyp >> (r + 1)), C), dim3(1024), 0, st, vertmap, extents, C,
                       seed, w3, r);
  }
  hipLaunchKernelGGL(k_p3d_finish, dim3(C), dim3(kFinThreads), 0, st, vertmap, extents, C, n_hyp, seed, nm_evals, w3, final_out,
                     poses_out, energy_out);
  if (eye_out &&
      hipMemcpyAsync(eye_out, w3.eye, (size_t)HW * 3 * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
    return PCNN_EHIP;
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
