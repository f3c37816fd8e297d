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
//   k_p2d_collect / k_p2d_count / k_p2d_select / k_p2d_finish: the 8 rounds
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

// attempt a of hypothesis h draws Philox4x32-10 blocks (draw / 4, h, 'P2D', a), words in order
struct Stream {
  uint32_t k0, k1, h, a, ctr;
  int word;
  U4 buf;
  __device__ Stream(uint64_t seed, uint32_t hyp, uint32_t attempt)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), h(hyp), a(attempt), ctr(0), word(4), buf{0, 0, 0, 0} {}
  __device__ uint32_t next() {
    if (word == 4) {
      buf = philox(U4{ctr++, h, 0x50324400u, a}, k0, k1);
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
  // 1e-13 of their root (the oracle stops at the same sweep: identical IEEE
  // double operations on both sides)
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
    if (mstep < 1e-13) break;
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

__global__ void __launch_bounds__(1024) k_p2d_subset(uint64_t seed, P2dWs ws) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int c = blockIdx.x, r = blockIdx.y, t = threadIdx.x, lane = pcnn::lane_id(), wave = t >> 6;
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
  const double q = 1.0 - (double)rate;
  int carry = 0;  // s_{j0}
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
    int wb = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
      if (w < wave) wb += wsum[w];
      tot += wsum[w];
    }
    const long pos = (long)carry + wb + incl - g;  // s_{j0 + t}
    if (pos < N) S[j0 + t] = (int)pos;
    if (pos < N && pos + g >= N) ws.subcnt[c * kRounds + r] = j0 + t + 1;  // the last index below N
    __syncthreads();  // wsum is rewritten by the next chunk
    if ((long)carry + tot >= N) break;  // block-uniform
    carry += tot;
  }
  (void)carry_s;
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
  Stream rs(seed, (uint32_t)h, (uint32_t)a);
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

// The first kAttempts attempts of every hypothesis at once, one lane each:
// the reference's loop runs attempts until one is accepted, and attempts are
// independent (each its own stream), so they need not wait for each other.
__global__ void __launch_bounds__(64) k_p2d_attempts(const float* __restrict__ vm, const float* __restrict__ ext,
                                                     int H, int W, int C, Cam k, uint64_t seed, int n_hyp, int T,
                                                     P2dWs ws) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_obj = *ws.nobj;
  if (id >= n_hyp * T || n_obj == 0) return;
  const int h = id % n_hyp, a = id / n_hyp;
  double* rec = ws.att + (size_t)(h * T + a) * kAttRec;
  int obj, px4[4];
  Pose P;
  if (!p2d_attempt(vm, ext, H, W, C, k, seed, h, a, n_obj, ws, obj, px4, P)) {
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
// stores it.  max_iter bounds the attempts (the reference: 10,000,000).
__global__ void __launch_bounds__(64) k_p2d_pick(const float* __restrict__ vm, const float* __restrict__ ext, int H,
                                                 int W, int C, Cam k, uint64_t seed, int n_hyp, int max_iter, int T,
                                                 P2dWs ws, float* __restrict__ hyps_out,
                                                 int32_t* __restrict__ hyp_px) {
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
      int o = -1, q4[4];
      Pose Q;
      const bool acc = a < max_iter && p2d_attempt(vm, ext, H, W, C, k, seed, h, a, n_obj, ws, o, q4, Q);
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
  for (int i = 0; i < 4; i++) hyp_px[h * 4 + i] = obj >= 0 ? px4[i] : -1;
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
// object keeps the better half (k_p2d_select); survivor lists live in the
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

__global__ void __launch_bounds__(256) k_p2d_count(const float* __restrict__ vm, const float* __restrict__ ext, int W,
                                                   int C, Cam k, P2dWs ws, int r, int32_t* __restrict__ inl_out) {
  __shared__ int part[4];
  const int j = blockIdx.x, oi = blockIdx.y;
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
  for (int i = threadIdx.x; i < ns; i += 256) {  // countInliers2D (:1171-1214)
    const int idx = L[S[i]];
    const double u0 = idx % W, v0 = idx / W;
    const F3 o = mode3d(vm, ext, C, obj, idx);
    double u, v;
    project(P, D3{o.x, o.y, o.z}, k, u, v);
    if (sqrt((u0 - u) * (u0 - u) + (v0 - v) * (v0 - v)) < 10.0f) cnt++;
  }
  cnt = pcnn::wave_sum(cnt);
  if (pcnn::lane_id() == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int c = part[0] + part[1] + part[2] + part[3];
    ws.rc[oi * kMaxHypBlock + j] = c;
    inl_out[h * kRounds + r] = c;
  }
}

// stable sort by inliers (descending, then list position), keep the better half
__global__ void __launch_bounds__(1024) k_p2d_select(P2dWs ws) {
  __shared__ int hl[kMaxHypBlock], hc[kMaxHypBlock], tmp[kMaxHypBlock];
  const int oi = blockIdx.x;
  if (oi >= *ws.nobj) return;
  const int m = ws.rm[oi];
  if (m <= 1) return;
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    hl[j] = ws.rl[oi * kMaxHypBlock + j];
    hc[j] = ws.rc[oi * kMaxHypBlock + j];
  }
  __syncthreads();
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

struct Layout {
  size_t colcnt, coloff, count, lists, listoff, objs, nobj, subcnt, hyp, att, rl, rc, rm, sub, total;
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
  hipLaunchKernelGGL(k_p2d_attempts, dim3((n_hyp * T + 63) / 64), dim3(64), 0, st, vertmap, extents, H, W, C, k, seed,
                     n_hyp, T, ws);
  hipLaunchKernelGGL(k_p2d_pick, dim3(n_hyp), dim3(64), 0, st, vertmap, extents, H, W, C, k, seed, n_hyp, max_iter, T,
                     ws, hyps_out, hyp_px);
  hipLaunchKernelGGL(k_p2d_collect, dim3(C), dim3(64), 0, st, n_hyp, ws);
  for (int r = 0; r < kRounds; r++) {
    const int gx = std::max(1, n_hyp >> r);  // survivors halve each round (one stays one)
    hipLaunchKernelGGL(k_p2d_count, dim3(gx, C), dim3(256), 0, st, vertmap, extents, W, C, k, ws, r, inl_out);
    hipLaunchKernelGGL(k_p2d_select, dim3(C), dim3(1024), 0, st, ws);
  }
  hipLaunchKernelGGL(k_p2d_finish, dim3(C), dim3(64), 0, st, C, n_hyp, ws, final_out, poses_out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
