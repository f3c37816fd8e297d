// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// RGB-only pose estimation of the reference's test-time path (SURVEY.md §8(f)
// row 4, RANSAC half): Synthesizer::estimatePose2D
// (lib/synthesize/synthesize.cpp:1571-1766), reached through
// synthesizer.pyx:74-82 estimate_poses_2d from lib/fcn/test.py:1364
// (cfg.TEST.VERTEX_REG_3D: the vertex map holds object coordinates scaled to
// [0, 1] by the class extents).  Restated pieces:
//   getLabels (:1010-1031, column-major traversal, > minArea = 400 px),
//   getBb3Ds / getBB3D (:1035-1048, detection.h:45-64),
//   getMode3D (:1052-1071), pointLineDistance (:1074-1080),
//   samplePoint2D (:1084-1104), hypothesis sampling (:1616-1688),
//   getBB2D (detection.h:78-109), the preemptive loop (:1693-1727) with
//   countInliers2D (:1171-1214: pixel skips max(1, G), G ~
//   negative_binomial(1, maxPixels / N), i.e. geometric -- see the RNG
//   choice below),
//   getWorkingQueue (:1150-1160), and the output layout (:1729-1764).
// Deliberate, documented choices (parity unpinned: OpenCV, NLopt absent):
//   * RNG: attempt a of hypothesis h draws from its own Philox4x32-10 stream
//     (key = seed, counter = (draw, h, 'P2D', a)), uniform ints by rejection;
//     h keeps its first accepted attempt (independent attempts: the GPU
//     evaluates a batch of them at once); the
//     reference's per-thread mt19937 streams (thread_rand.cpp) are assigned
//     to hypotheses by the OpenMP schedule, i.e. nondeterministically.
//   * The rounds' pixel subsets: the reference draws G from a default-seeded
//     std::mt19937 per countInliers2D call (the same subset for every
//     hypothesis of a round).  Here G_j of round r of class c comes from the
//     Philox4x32-10 block (j, c, 'SUB0' + r, 0) under key seed: U =
//     (x 2^21 + (y >> 11) + 0.5) 2^-53 from its first two words and G = the
//     largest k with U < q^k, q = 1 - p (inverse CDF of the geometric law
//     on repeated double products, bit-reproducible on the GPU).  Same
//     distribution; the draws themselves are unpinned (round 5: the host
//     replay of libstdc++'s negative_binomial pinned nothing, because the
//     hypotheses already come from Philox streams).
//   * Hypotheses are stored in ascending h (the reference appends in
//     completion order under omp critical); the per-round sort is stable
//     (inliers descending, then h): one legal order of std::sort's ties.
//   * cv::solvePnP(CV_P3P) is restated as Grunert's P3P (distance ratios
//     u = s2/s1, v = s3/s1; the quartic in v from eliminating u, its roots by
//     Durand-Kerner sweeps until the steps fall below 1e-9 of their roots,
//     polished by 4 Newton steps -- the real roots come out the same as with
//     a 1e-13 stop, which 2/3 of the quartics never reach: their clustered
//     roots leave the sweeps oscillating at 1e-13..1e-10), the camera-frame
//     triangle aligned to the model triangle by orthonormal triads, and the
//     solution whose reprojection of the 4th point is closest kept -- as
//     OpenCV's p3p.cpp selects it.
//   * The preemptive "refinement" in estimatePose2D calls updateHyp3D
//     (:1722), which returns at once in the 2-D path (inlierPts -- the 3-D
//     correspondences -- stay empty, :1374), and refineWithOpt's optEnergy2D
//     divides by that empty list's size (:1457): every energy is inf or NaN,
//     so NLopt keeps the start point.  The final pose is therefore the winning
//     hypothesis's P3P pose; both steps are restated as the identity.
//   * The sampling loop is capped at max_iter draws per hypothesis (the
//     reference: 10,000,000).
#include "orc_common.h"
#include <algorithm>
#include <complex>
#include <random>
#include <vector>

namespace {

// ---- Philox4x32-10 (Salmon et al., SC'11; Random123 constants) -------------
struct U4 { uint32_t v[4]; };
U4 philox(U4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0], p1 = (uint64_t)0xCD9E8D57u * c.v[2];
    U4 o;
    o.v[0] = (uint32_t)(p1 >> 32) ^ c.v[1] ^ k0;
    o.v[1] = (uint32_t)p1;
    o.v[2] = (uint32_t)(p0 >> 32) ^ c.v[3] ^ k1;
    o.v[3] = (uint32_t)p0;
    c = o;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// max(1, G) of one pixel skip (see the RNG notes above; the GPU's p2d_gap)
int subset_gap(uint64_t seed, int c, int r, int j, double q) {
  const U4 b = philox(U4{{(uint32_t)j, (uint32_t)c, 0x53554230u + (uint32_t)r, 0u}}, (uint32_t)seed,
                      (uint32_t)(seed >> 32));
  const double U = ((double)b.v[0] * 2097152.0 + (double)(b.v[1] >> 11) + 0.5) * 0x1p-53;
  int k = 0;
  double t = q;
  while (t > U) {
    k++;
    t = t * q;
  }
  return k > 1 ? k : 1;
}

struct Stream {
  uint32_t k0, k1, h, a, ctr = 0;
  int word = 4;
  U4 buf;
  Stream(uint64_t seed, uint32_t hyp, uint32_t attempt)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), h(hyp), a(attempt) {}
  uint32_t next() {
    if (word == 4) {
      buf = philox(U4{{ctr++, h, 0x50324400u, a}}, k0, k1);
      word = 0;
    }
    return buf.v[word++];
  }
  // uniform in [0, n): reject the top 2^32 mod n values
  int uniform(int n) {
    const uint32_t un = (uint32_t)n;
    const uint32_t lim = (uint32_t)(0x100000000ull - (0x100000000ull % un));
    uint32_t x;
    do { x = next(); } while (lim != 0 && x >= lim);
    return (int)(x % un);
  }
};

struct V3 { double x, y, z; };
V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double nrm(V3 a) { return std::sqrt(dot(a, a)); }

struct F3 { float x, y, z; };  // cv::Point3f

struct Pose { double R[9]; double t[3]; };

struct Cam { double fx, fy, px, py; };

// cv::projectPoints without distortion (OpenCV's cvProjectPoints2 order)
void project(const Pose& P, V3 X, const Cam& k, double& u, double& v) {
  const double* R = P.R;
  const double x = R[0] * X.x + R[1] * X.y + R[2] * X.z + P.t[0];
  const double y = R[3] * X.x + R[4] * X.y + R[5] * X.z + P.t[1];
  double z = R[6] * X.x + R[7] * X.y + R[8] * X.z + P.t[2];
  z = z != 0.0 ? 1.0 / z : 1.0;
  u = x * z * k.fx + k.px;
  v = y * z * k.fy + k.py;
}

// getMode3D (synthesize.cpp:1052-1071): the object coordinate of pixel p
F3 mode3d(const float* vertmap, const float* extents, int C, int objID, int p) {
  const float* m = vertmap + (size_t)p * 3 * C + 3 * objID;
  float o[3];
  for (int i = 0; i < 3; i++) {
    const float vmin = -extents[objID * 3 + i] / 2, vmax = extents[objID * 3 + i] / 2;
    const float a = (float)(1.0 / (double)(vmax - vmin));
    const float b = (float)(-1.0 * (double)vmin / (double)(vmax - vmin));
    o[i] = (m[i] - b) / a;
  }
  return {o[0], o[1], o[2]};
}

double norm3f(F3 a, F3 b) {  // cv::norm(Point3f - Point3f)
  const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return std::sqrt((double)dx * dx + (double)dy * dy + (double)dz * dz);
}

double point_line(F3 p1, F3 p2, F3 p3) {  // :1074-1080, float vector ops, double norms
  const F3 a{p2.x - p1.x, p2.y - p1.y, p2.z - p1.z}, b{p3.x - p1.x, p3.y - p1.y, p3.z - p1.z};
  const F3 c{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  const double nc = std::sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z);
  const double na = std::sqrt((double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z);
  return nc / na;
}

// ---- Grunert's P3P ----------------------------------------------------------
// real roots of c[4] v^4 + ... + c[0]
int quartic_roots(const double* c, double* out) {
  const double a4 = c[4];
  double mx = 0;
  for (int i = 0; i < 4; i++) mx = std::max(mx, std::fabs(c[i]));
  if (!(std::fabs(a4) > 1e-12 * mx)) return 0;
  double a[4];
  for (int i = 0; i < 4; i++) a[i] = c[i] / a4;
  double bound = 1;
  for (int i = 0; i < 4; i++) bound = std::max(bound, 1 + std::fabs(a[i]));
  typedef std::complex<double> cd;
  cd z[4];
  const cd seed(0.4, 0.9);
  cd w(1, 0);
  for (int k = 0; k < 4; k++) { z[k] = w * bound; w *= seed; }
  auto pe = [&](cd x) { return (((x + a[3]) * x + a[2]) * x + a[1]) * x + a[0]; };
  // up to 200 sweeps, stopping at the first whose steps are all below 1e-9
  // of their root (pose2d.hip stops at the same sweep)
  for (int it = 0; it < 200; it++) {
    double mstep = 0;
    for (int k = 0; k < 4; k++) {
      cd den(1, 0);
      for (int j = 0; j < 4; j++)
        if (j != k) den *= (z[k] - z[j]);
      if (den == cd(0, 0)) continue;
      const cd st = pe(z[k]) / den;
      z[k] -= st;
      mstep = std::max(mstep, (std::fabs(st.real()) + std::fabs(st.imag())) /
                                  (1 + std::fabs(z[k].real()) + std::fabs(z[k].imag())));
    }
    if (mstep < 1e-9) break;
  }
  int n = 0;
  for (int k = 0; k < 4; k++) {
    if (!(std::fabs(z[k].imag()) <= 1e-6 * (1 + std::abs(z[k])))) continue;
    double x = z[k].real();
    for (int it = 0; it < 4; it++) {  // Newton polish on the real quartic
      const double p = (((x + a[3]) * x + a[2]) * x + a[1]) * x + a[0];
      const double dp = ((4 * x + 3 * a[3]) * x + 2 * a[2]) * x + a[1];
      if (dp == 0) break;
      x -= p / dp;
    }
    out[n++] = x;
  }
  return n;
}

void polymul(const double* a, int na, const double* b, int nb, double* out) {  // coefficient arrays, low first
  for (int i = 0; i < na + nb - 1; i++) out[i] = 0;
  for (int i = 0; i < na; i++)
    for (int j = 0; j < nb; j++) out[i + j] += a[i] * b[j];
}

// Triad alignment of the model triangle P onto the camera-frame triangle Q
Pose triad(const V3* P, const V3* Q) {
  auto frame = [](const V3* X, V3* e) {
    e[0] = (1.0 / nrm(X[1] - X[0])) * (X[1] - X[0]);
    V3 w = X[2] - X[0];
    w = w - dot(w, e[0]) * e[0];
    e[1] = (1.0 / nrm(w)) * w;
    e[2] = cross(e[0], e[1]);
  };
  V3 e[3], f[3];
  frame(P, e);
  frame(Q, f);
  Pose o;
  const double fe[3][3] = {{f[0].x, f[1].x, f[2].x}, {f[0].y, f[1].y, f[2].y}, {f[0].z, f[1].z, f[2].z}};
  const double ee[3][3] = {{e[0].x, e[1].x, e[2].x}, {e[0].y, e[1].y, e[2].y}, {e[0].z, e[1].z, e[2].z}};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) o.R[3 * r + c] = fe[r][0] * ee[c][0] + fe[r][1] * ee[c][1] + fe[r][2] * ee[c][2];
  const V3 RP{o.R[0] * P[0].x + o.R[1] * P[0].y + o.R[2] * P[0].z, o.R[3] * P[0].x + o.R[4] * P[0].y + o.R[5] * P[0].z,
              o.R[6] * P[0].x + o.R[7] * P[0].y + o.R[8] * P[0].z};
  o.t[0] = Q[0].x - RP.x;
  o.t[1] = Q[0].y - RP.y;
  o.t[2] = Q[0].z - RP.z;
  return o;
}

// solvePnP(..., CV_P3P) on 4 correspondences: solve with points 0-2, keep the
// solution whose reprojection of point 3 is closest
bool p3p(const F3* X, const float (*m)[2], const Cam& k, Pose& best) {
  V3 P[4], j[4];
  for (int i = 0; i < 4; i++) {
    P[i] = {X[i].x, X[i].y, X[i].z};
    const V3 r{((double)m[i][0] - k.px) / k.fx, ((double)m[i][1] - k.py) / k.fy, 1.0};
    j[i] = (1.0 / nrm(r)) * r;
  }
  const double a = nrm(P[1] - P[2]), b = nrm(P[0] - P[2]), c = nrm(P[0] - P[1]);
  const double ca = dot(j[1], j[2]), cb = dot(j[0], j[2]), cg = dot(j[0], j[1]);
  const double a2 = a * a, b2 = b * b, c2 = c * c;
  if (!(b2 > 0)) return false;
  const double K1 = (a2 - c2) / b2, Kc = c2 / b2;
  const double Nv[3] = {1 + K1, -2 * K1 * cb, K1 - 1};  // u * D(v) = N(v)
  const double Dv[2] = {2 * cg, -2 * ca};
  const double qv[3] = {1 - Kc, 2 * Kc * cb, -Kc};       // 1 - (c^2/b^2)(1 + v^2 - 2 v cos b)
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
    if (std::fabs(D) < 1e-12) continue;
    const double u = ((K1 - 1) * v * v - 2 * K1 * cb * v + 1 + K1) / D;
    const double q = 1 + v * v - 2 * v * cb;
    if (!(q > 0) || !(u > 0) || !(v > 0)) continue;
    const double s1 = std::sqrt(b2 / q);
    const V3 Q[3] = {s1 * j[0], (u * s1) * j[1], (v * s1) * j[2]};
    const Pose cand = triad(P, Q);
    double pu, pv;
    project(cand, P[3], k, pu, pv);
    const double e = (pu - m[3][0]) * (pu - m[3][0]) + (pv - m[3][1]) * (pv - m[3][1]);
    if (!(e == e)) continue;
    if (best_err < 0 || e < best_err) { best_err = e; best = cand; }
  }
  return best_err >= 0;
}

// getBB2D (detection.h:78-109) area: float projections, int truncation, clamp
int bb_area(const Pose& P, const F3* bb3, const Cam& k, int W, int H) {
  int minX = W - 1, maxX = 0, minY = H - 1, maxY = 0;
  for (int i = 0; i < 8; i++) {
    double u, v;
    project(P, {bb3[i].x, bb3[i].y, bb3[i].z}, k, u, v);
    const float fu = (float)u, fv = (float)v;
    minX = orc::f2i_sat(std::min((float)minX, fu));
    minY = orc::f2i_sat(std::min((float)minY, fv));
    maxX = orc::f2i_sat(std::max((float)maxX, fu));
    maxY = orc::f2i_sat(std::max((float)maxY, fv));
  }
  auto cl = [](int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); };
  minX = cl(minX, 0, W - 1); maxX = cl(maxX, 0, W - 1);
  minY = cl(minY, 0, H - 1); maxY = cl(maxY, 0, H - 1);
  return (maxX - minX + 1) * (maxY - minY + 1);
}

struct Hyp { int h, obj, inliers = 0; Pose pose; };

}  // namespace

// hyps_out (n_hyp, 13): [objID (or -1), R (9, row-major), t (3)]; hyp_px (n_hyp, 4)
// sampled pixel indices; inl_out (n_hyp, 8) inlier count of each preemptive
// round (-1 when the hypothesis was no longer in the queue); final_out (C, 3)
// [h, inliers, hypotheses of the class] of the surviving hypothesis (-1 when
// none); poses_out (3, 4, C) the reference's output layout.  Returns the
// number of classes that took part (object_ids).
ORC_API int orc_pose2d(const int* label, const float* vertmap, const float* extents, int H, int W, int C, float fx,
                       float fy, float px, float py, uint64_t seed, int n_hyp, int max_iter, float* poses_out,
                       float* hyps_out, int* hyp_px, int* inl_out, int* final_out) {
  const Cam k{fx, fy, px, py};
  std::vector<std::vector<int>> labels(C);
  for (int x = 0; x < W; x++)
    for (int y = 0; y < H; y++) labels[label[y * W + x]].push_back(y * W + x);
  std::vector<int> objs;
  for (int c = 1; c < C; c++)
    if ((float)labels[c].size() > 400.0f) objs.push_back(c);
  for (int i = 0; i < n_hyp * 13; i++) hyps_out[i] = 0;
  for (int i = 0; i < n_hyp; i++) hyps_out[i * 13] = -1;
  for (int i = 0; i < n_hyp * 4; i++) hyp_px[i] = -1;
  for (int i = 0; i < n_hyp * 8; i++) inl_out[i] = -1;
  for (int i = 0; i < C * 3; i++) final_out[i] = -1;
  if (objs.empty()) return 0;
  std::vector<std::vector<Hyp>> hypmap(C);
  for (int h = 0; h < n_hyp; h++) {
    for (int it = 0; it < max_iter; it++) {
      Stream rs(seed, (uint32_t)h, (uint32_t)it);  // attempt it of hypothesis h draws from its own stream
      const int obj = objs[rs.uniform((int)objs.size())];
      const auto& L = labels[obj];
      float m[4][2];
      F3 X[4];
      int px4[4], n = 0;
      bool ok = true;
      for (int s = 0; s < 4 && ok; s++) {  // samplePoint2D x 4
        const int idx = L[rs.uniform((int)L.size())];
        const float u = (float)(idx % W), v = (float)(idx / W);
        double md = -1;
        for (int q = 0; q < n; q++) {
          const float dx = m[q][0] - u, dy = m[q][1] - v;
          const double d = std::sqrt((double)dx * dx + (double)dy * dy);
          md = md < 0 ? d : std::min(md, d);
        }
        if (md > 0 && md < 10) { ok = false; break; }
        const F3 o = mode3d(vertmap, extents, C, obj, idx);
        if (o.x == 0 && o.y == 0 && o.z == 0) { ok = false; break; }
        md = -1;
        for (int q = 0; q < n; q++) {
          const double d = norm3f(X[q], o);
          md = md < 0 ? d : std::min(md, d);
        }
        if (md > 0 && md < 0.01) { ok = false; break; }
        m[n][0] = u; m[n][1] = v; X[n] = o; px4[n] = idx; n++;
      }
      if (!ok) continue;
      if (point_line(X[0], X[1], X[2]) < 0.01 || point_line(X[0], X[1], X[3]) < 0.01 ||
          point_line(X[0], X[2], X[3]) < 0.01 || point_line(X[1], X[2], X[3]) < 0.01)
        continue;
      Pose P;
      if (!p3p(X, m, k, P)) continue;
      bool out = false;
      for (int q = 0; q < 4 && !out; q++) {
        double u, v;
        project(P, {X[q].x, X[q].y, X[q].z}, k, u, v);
        const float du = m[q][0] - (float)u, dv = m[q][1] - (float)v;  // Point2f difference
        if (!(std::sqrt((double)du * du + (double)dv * dv) < 10)) out = true;
      }
      if (out) continue;
      const float e0 = extents[obj * 3] * 0.5f, e1 = extents[obj * 3 + 1] * 0.5f, e2 = extents[obj * 3 + 2] * 0.5f;
      const F3 bb3[8] = {{e0, e1, e2}, {-e0, e1, e2}, {e0, -e1, e2}, {-e0, -e1, e2},
                         {e0, e1, -e2}, {-e0, e1, -e2}, {e0, -e1, -e2}, {-e0, -e1, -e2}};
      if ((float)bb_area(P, bb3, k, W, H) < 400.0f) continue;
      Hyp hy;
      hy.h = h; hy.obj = obj; hy.pose = P;
      hypmap[obj].push_back(hy);
      hyps_out[h * 13] = (float)obj;
      for (int i = 0; i < 9; i++) hyps_out[h * 13 + 1 + i] = (float)P.R[i];
      for (int i = 0; i < 3; i++) hyps_out[h * 13 + 10 + i] = (float)P.t[i];
      for (int i = 0; i < 4; i++) hyp_px[h * 4 + i] = px4[i];
      break;
    }
  }
  // preemptive loop: every class runs 8 rounds (<= 256 hypotheses halve to
  // one in at most 8; a lone hypothesis is counted until refSteps reaches 8)
  for (int c = 0; c < C; c++) {
    auto& hs = hypmap[c];
    if (hs.empty()) continue;
    const auto& L = labels[c];
    const int N = (int)L.size();
    for (int round = 1; round <= 8; round++) {
      const int maxPixels = 1000 * round;
      const float rate = maxPixels / (float)N;  // :1191
      std::vector<int> sub;
      const double q = 1.0 - (double)rate;
      for (int i = 0, j = 0; i < N; j++) {
        sub.push_back(i);
        if (rate < 1) i += subset_gap(seed, c, round - 1, j, q);
        else i++;
      }
      for (auto& hy : hs) {
        int cnt = 0;
        for (int i : sub) {
          const int idx = L[i];
          const double u0 = idx % W, v0 = idx / W;
          const F3 o = mode3d(vertmap, extents, C, c, idx);
          double u, v;
          project(hy.pose, {o.x, o.y, o.z}, k, u, v);
          if (std::sqrt((u0 - u) * (u0 - u) + (v0 - v) * (v0 - v)) < 10.0f) cnt++;
        }
        hy.inliers = cnt;
        inl_out[hy.h * 8 + round - 1] = cnt;
      }
      if (hs.size() > 1) {
        std::stable_sort(hs.begin(), hs.end(), [](const Hyp& a, const Hyp& b) { return a.inliers > b.inliers; });
        hs.erase(hs.begin() + hs.size() / 2, hs.end());
      }
    }
    const Hyp& w = hs[0];
    final_out[c * 3] = w.h;
    final_out[c * 3 + 1] = w.inliers;
    int nh = 0;
    for (int h = 0; h < n_hyp; h++) nh += hyps_out[h * 13] == (float)c;
    final_out[c * 3 + 2] = nh;
    for (int y = 0; y < 3; y++)
      for (int x = 0; x < 4; x++)
        poses_out[c + C * (y * 4 + x)] = x < 3 ? (float)w.pose.R[y * 3 + x] : (float)w.pose.t[y];
  }
  return (int)objs.size();
}

// ===========================================================================
// Depth-based pose estimation: Synthesizer::estimatePose3D
// (lib/synthesize/synthesize.cpp:1769-1965), reached through synthesizer.pyx:
// 86-95 estimate_poses_3d from lib/fcn/test.py:1385 (cfg.TEST.VERTEX_REG_3D;
// its poses then go to refine_poses, test.py:1403-1416).  Restated pieces:
//   getEye / pxToEye (:1383-1410): camera coordinates of the depth map;
//   getLabels (as estimatePose2D), samplePoint3D (:1105-1134) x 3,
//   Hypothesis(pts3D) = calcRigidBodyTransform (Hypothesis.cpp:178-246:
//   centroids, the 3x3 covariance, SVD, the sign fix, R = V D U^T,
//   t = cB - R cA), the reconstruction check (< 1 cm), getBB2D area >= 400;
//   the preemptive loop (:1889-1926) with countInliers3D (:1227-1280: depth
//   holes step to the next pixel without a draw; inliers < 1 cm), the stable
//   halving, updateHyp3D (:1347-1370: >= 4 inliers, filterInliers3D
//   (:1308-1322) then the refit); the final refineWithOpt(.., 100, is_3D)
//   (:1510-1567) over optEnergy3D (:1464-1507) when inliers > 10, and the
//   output layout (:1941-1963).
// Deliberate, documented choices (parity unpinned: OpenCV, NLopt absent):
//   * RNG: Philox streams as estimatePose2D: attempt a of hypothesis h on
//     (draw, h, 'P3D', a); the rounds' pixel skips on (j, class, 'SUB0' + r)
//     with the inverse-CDF geometric law of the 2-D restatement (the same
//     streams); filterInliers3D's picks (irand with replacement) on
//     (draw, h, 'F3D', 1024 r + k) for pick k, r = the round (0-7) or 8 for
//     the final filter.
//   * cv::SVD of the covariance is restated as a one-sided Jacobi (fixed
//     pivot order, rotations skipped below 1e-15 relative, at most 16
//     sweeps), singular values sorted descending, the third left vector the
//     cross product of the first two when its singular value is below 1e-9 of
//     the first (three-point covariances have rank two): R = V D U^T does
//     not depend on the SVD's sign conventions.  The centroid and covariance
//     sums, and optEnergy3D's float sum, run in the GPU workgroup's fixed
//     tree (tree1024; the reference's loops are sequential).
//   * sin, cos, acos (Rodrigues) from + - * / sqrt only (dsincos, dacos), so
//     the GPU reproduces them bit for bit; libm differs in the last ulp.
//   * Hypothesis poses stay (R, t) between steps; the reference round-trips
//     them through Rodrigues vectors (our2cv / cv2our), a change at rounding
//     level.
//   * refineWithOpt's NLopt LN_NELDERMEAD is the bounded Nelder-Mead of
//     posecnn_amd/synthesize/icp.py nelder_mead_steps (6 parameters: Rodrigues
//     vector and translation, +-10 deg / +-0.1 / +-0.1 / +-0.5 m bounds, 100
//     evaluations).
namespace {

struct TStream {  // Philox words of the stream (draw, h, tag, a)
  uint32_t k0, k1, h, tag, a, ctr = 0;
  int word = 4;
  U4 buf;
  TStream(uint64_t seed, uint32_t hyp, uint32_t tg, uint32_t attempt)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), h(hyp), tag(tg), a(attempt) {}
  uint32_t next() {
    if (word == 4) {
      buf = philox(U4{{ctr++, h, tag, a}}, k0, k1);
      word = 0;
    }
    return buf.v[word++];
  }
  int uniform(int n) {
    const uint32_t un = (uint32_t)n;
    const uint32_t lim = (uint32_t)(0x100000000ull - (0x100000000ull % un));
    uint32_t x;
    do { x = next(); } while (lim != 0 && x >= lim);
    return (int)(x % un);
  }
};
constexpr uint32_t kTagP3D = 0x50334400u, kTagF3D = 0x46334400u;

// one-sided Jacobi SVD of a 3x3 (row-major): A = U diag(S) V^T, S descending
void svd3(const double* A, double* U, double* S, double* V) {
  double M[9], Vm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int i = 0; i < 9; i++) M[i] = A[i];
  const int pq[3][2] = {{0, 1}, {0, 2}, {1, 2}};
  for (int sweep = 0; sweep < 16; sweep++) {
    bool rot = false;
    for (int k = 0; k < 3; k++) {
      const int p = pq[k][0], q = pq[k][1];
      double al = 0, be = 0, ga = 0;
      for (int r = 0; r < 3; r++) {
        al = al + M[r * 3 + p] * M[r * 3 + p];
        be = be + M[r * 3 + q] * M[r * 3 + q];
        ga = ga + M[r * 3 + p] * M[r * 3 + q];
      }
      if (ga == 0.0 || std::fabs(ga) <= 1e-15 * std::sqrt(al * be)) continue;
      const double zeta = (be - al) / (2.0 * ga);
      const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
      const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
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
    sv[i] = std::sqrt(a);
  }
  int o[3] = {0, 1, 2};  // descending, stable
  for (int i = 1; i < 3; i++)
    for (int j = i; j > 0 && sv[o[j]] > sv[o[j - 1]]; j--) std::swap(o[j], o[j - 1]);
  for (int k = 0; k < 3; k++) {
    S[k] = sv[o[k]];
    for (int r = 0; r < 3; r++) {
      V[r * 3 + k] = Vm[r * 3 + o[k]];
      U[r * 3 + k] = S[k] > 0 ? M[r * 3 + o[k]] / S[k] : 0.0;
    }
  }
  if (!(S[2] > 1e-9 * S[0])) {  // rank two: complete U
    U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
    U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
    U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
  }
}

double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// The fixed summation tree of the GPU's 1024-thread workgroups (n <= 1024):
// leaf i = 0.0 + x_i (0.0 past n); each 64-leaf wave folds by halving
// (p_i += p_{i + off}, off = 32 .. 1), then the 16 wave sums fold the same way
// (off = 8 .. 1) -- posecnn_amd/csrc/pose2d.hip tree_sum
template <class T, class F>
T tree1024(F x, int n) {
  T p[1024];
  for (int i = 0; i < 1024; i++) p[i] = i < n ? (T)0 + x(i) : (T)0;
  T w[16];
  for (int v = 0; v < 16; v++) {
    T* q = p + 64 * v;
    for (int off = 32; off >= 1; off >>= 1)
      for (int i = 0; i < off; i++) q[i] = q[i] + q[i + off];
    w[v] = q[0];
  }
  for (int off = 8; off >= 1; off >>= 1)
    for (int i = 0; i < off; i++) w[i] = w[i] + w[i + off];
  return w[0];
}
template <class F>
double tsum(F x, int n) { return tree1024<double>(x, n); }

// calcRigidBodyTransform (Hypothesis.cpp:186-241): b ~ R a + t.  The
// centroid and covariance sums in tree1024 order (OpenCV: sequential).
Pose kabsch(const V3* a, const V3* b, int n) {
  const double inv = 1.0 / (double)n;
  const V3 cA{tsum([&](int i) { return a[i].x; }, n) * inv, tsum([&](int i) { return a[i].y; }, n) * inv,
              tsum([&](int i) { return a[i].z; }, n) * inv};
  const V3 cB{tsum([&](int i) { return b[i].x; }, n) * inv, tsum([&](int i) { return b[i].y; }, n) * inv,
              tsum([&](int i) { return b[i].z; }, n) * inv};
  double H[9];  // pointsA * pointsB^T
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      H[r * 3 + c] = tsum(
          [&](int i) {
            const double pa = r == 0 ? a[i].x - cA.x : r == 1 ? a[i].y - cA.y : a[i].z - cA.z;
            const double pb = c == 0 ? b[i].x - cB.x : c == 1 ? b[i].y - cB.y : b[i].z - cB.z;
            return pa * pb;
          },
          n);
  double U[9], S[3], V[9];
  svd3(H, U, S, V);
  double VU[9];  // V U^T
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) VU[r * 3 + c] = V[r * 3 + 0] * U[c * 3 + 0] + V[r * 3 + 1] * U[c * 3 + 1] + V[r * 3 + 2] * U[c * 3 + 2];
  const double sg = det3(VU) < 0 ? -1.0 : 1.0;
  Pose P;
  for (int r = 0; r < 3; r++)  // V diag(1, 1, sg) U^T
    for (int c = 0; c < 3; c++)
      P.R[r * 3 + c] = V[r * 3 + 0] * U[c * 3 + 0] + V[r * 3 + 1] * U[c * 3 + 1] + (V[r * 3 + 2] * sg) * U[c * 3 + 2];
  const double ca[3] = {cA.x, cA.y, cA.z}, cb[3] = {cB.x, cB.y, cB.z};
  for (int r = 0; r < 3; r++) P.t[r] = -(P.R[r * 3 + 0] * ca[0] + P.R[r * 3 + 1] * ca[1] + P.R[r * 3 + 2] * ca[2]) + cb[r];
  return P;
}

V3 xform(const Pose& P, V3 p) {  // Hypothesis::transform
  return {P.R[0] * p.x + P.R[1] * p.y + P.R[2] * p.z + P.t[0], P.R[3] * p.x + P.R[4] * p.y + P.R[5] * p.z + P.t[1],
          P.R[6] * p.x + P.R[7] * p.y + P.R[8] * p.z + P.t[2]};
}

// sin / cos / acos from + - * / and sqrt only, so that the device computes
// the same bits (posecnn_amd/csrc/pose2d.hip): quadrant reduction by a
// two-part pi/2, the fdlibm kernel polynomials; acos by the half-angle
// identity and 6 Newton steps on asin
void dsincos(double x, double& s, double& c) {
  const double n = std::floor(x * 0.63661977236758134308 + 0.5);
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

double dasin_small(double x) {  // |x| <= sqrt(1/2)
  double y = x;
  for (int i = 0; i < 6; i++) {
    double s, c;
    dsincos(y, s, c);
    y = y - (s - x) / c;
  }
  return y;
}

double dacos(double c) {  // c in [-1, 1]
  if (c >= 0) return 2.0 * dasin_small(std::sqrt((1.0 - c) * 0.5));
  return 3.14159265358979311600 - 2.0 * dasin_small(std::sqrt((1.0 + c) * 0.5));
}

// cv::Rodrigues, vector -> matrix
void rod_v2m(const double* r, double* R) {
  const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
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

// cv::Rodrigues, matrix -> vector (cvRodrigues2 without its SVD re-orthonormalisation)
void rod_m2v(const double* R, double* r) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double th = dacos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double t = (R[0] + 1) * 0.5;
      rx = std::sqrt(std::max(t, 0.));
      t = (R[4] + 1) * 0.5;
      ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5;
      rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      th /= std::sqrt(rx * rx + ry * ry + rz * rz);
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

struct Corr { F3 obj, eye; };  // an inlier correspondence (obj coordinate, camera coordinate)

// filterInliers3D (:1308-1322): at least maxInliers -> maxInliers picks with
// replacement; pick k of round r draws from its own stream (draw, h, 'F3D',
// 1024 r + k), so the picks are independent of each other
std::vector<Corr> filter3d(const std::vector<Corr>& in, uint64_t seed, int h, int r) {
  if ((int)in.size() < 1000) return in;
  std::vector<Corr> out;
  for (int k = 0; k < 1000; k++) {
    TStream rs(seed, (uint32_t)h, kTagF3D, (uint32_t)(1024 * r + k));
    out.push_back(in[rs.uniform((int)in.size())]);
  }
  return out;
}

Pose kabsch_corr(const std::vector<Corr>& v) {
  std::vector<V3> a(v.size()), b(v.size());
  for (size_t i = 0; i < v.size(); i++) {
    a[i] = {v[i].obj.x, v[i].obj.y, v[i].obj.z};
    b[i] = {v[i].eye.x, v[i].eye.y, v[i].eye.z};
  }
  return kabsch(a.data(), b.data(), (int)v.size());
}

// optEnergy3D (:1464-1507): mean distance of the transformed object
// coordinates to the camera coordinates; the float sum of the double
// distances (each rounded to float) in tree1024 order (the reference: a
// sequential float accumulator)
double energy3d(const double* x, const std::vector<Corr>& v) {
  double Rd[9];
  rod_v2m(x, Rd);
  float Rf[9];
  for (int i = 0; i < 9; i++) Rf[i] = (float)Rd[i];  // jp::double2float
  const float tot = tree1024<float>(
      [&](int i) {
        const F3 o = v[i].obj;
        float tr[3];
        for (int r = 0; r < 3; r++) {
          const float m = Rf[r * 3 + 0] * o.x + Rf[r * 3 + 1] * o.y + Rf[r * 3 + 2] * o.z;
          tr[r] = (float)((double)m + x[3 + r]);
        }
        const double dx = (double)tr[0] - (double)v[i].eye.x, dy = (double)tr[1] - (double)v[i].eye.y,
                     dz = (double)tr[2] - (double)v[i].eye.z;
        return (float)std::sqrt(dx * dx + dy * dy + dz * dz);
      },
      (int)v.size());
  return (double)(tot / (float)v.size());
}

// the bounded Nelder-Mead of icp.py nelder_mead_steps (n parameters)
template <class F>
void nelder_mead(F f, int n, const double* x0, const double* lb, const double* ub, int max_eval, double* xbest,
                 double* fbest) {
  std::vector<std::vector<double>> pts(n + 1, std::vector<double>(x0, x0 + n));
  std::vector<double> vals(n + 1);
  for (int i = 0; i < n; i++) {
    const double st = std::min(0.25 * (ub[i] - lb[i]), std::min(0.75 * (ub[i] - x0[i]), 0.75 * (x0[i] - lb[i])));
    pts[i + 1][i] = x0[i] + st;
    for (int e = 0; e < n; e++)
      if (e != i) pts[i + 1][e] = x0[e] + 0.0;
  }
  for (int i = 0; i <= n; i++) vals[i] = f(pts[i].data());
  int nev = n + 1;
  auto clamp = [&](int e, double v) { return std::min(std::max(v, lb[e]), ub[e]); };
  std::vector<double> c(n), xr(n), xe(n), xc(n);
  while (nev < max_eval) {
    for (int i = 1; i <= n; i++)
      for (int j = i; j > 0 && vals[j] < vals[j - 1]; j--) {
        std::swap(vals[j], vals[j - 1]);
        std::swap(pts[j], pts[j - 1]);
      }
    for (int e = 0; e < n; e++) {
      double s = pts[0][e];
      for (int i = 1; i < n; i++) s = s + pts[i][e];
      c[e] = s / (double)n;
    }
    for (int e = 0; e < n; e++) xr[e] = clamp(e, c[e] + (c[e] - pts[n][e]));
    const double fr = f(xr.data());
    nev++;
    if (fr < vals[0] && nev < max_eval) {
      for (int e = 0; e < n; e++) xe[e] = clamp(e, c[e] + 2.0 * (c[e] - pts[n][e]));
      const double fe = f(xe.data());
      nev++;
      if (fe < fr) { pts[n] = xe; vals[n] = fe; } else { pts[n] = xr; vals[n] = fr; }
    } else if (fr < vals[n - 1]) {
      pts[n] = xr;
      vals[n] = fr;
    } else if (nev < max_eval) {
      for (int e = 0; e < n; e++)
        xc[e] = fr >= vals[n] ? clamp(e, c[e] + 0.5 * (pts[n][e] - c[e])) : clamp(e, c[e] + 0.5 * (xr[e] - c[e]));
      const double fc = f(xc.data());
      nev++;
      if (fc < std::min(fr, vals[n])) {
        pts[n] = xc;
        vals[n] = fc;
      } else {
        const int m = std::min(n, max_eval - nev);
        for (int i = 1; i <= m; i++) {
          for (int e = 0; e < n; e++) pts[i][e] = clamp(e, pts[0][e] + 0.5 * (pts[i][e] - pts[0][e]));
          vals[i] = f(pts[i].data());
        }
        nev += m > 0 ? m : 0;
      }
    }
  }
  int b = 0;
  for (int i = 1; i <= n; i++)
    if (vals[i] < vals[b]) b = i;
  for (int e = 0; e < n; e++) xbest[e] = pts[b][e];
  *fbest = vals[b];
}

struct Hyp3 { int h, obj, inliers = 0; Pose pose; std::vector<Corr> corr; };

}  // namespace

// eye_out (H, W, 3) camera coordinates; hyps_out (n_hyp, 13) [objID | R | t];
// hyp_px (n_hyp, 3); inl_out (n_hyp, 8) inliers per round (-1 not queued);
// final_out (C, 3) [h, inliers, hypotheses]; energy_out (C) optEnergy3D at the
// refined pose (0 when not refined); poses_out (3, 4, C).  Returns n objects.
ORC_API int orc_pose3d(const int* label, const uint16_t* depth, const float* vertmap, const float* extents, int H,
                       int W, int C, float fx, float fy, float px, float py, float depth_factor, uint64_t seed,
                       int n_hyp, int max_iter, int nm_evals, float* poses_out, float* eye_out, float* hyps_out,
                       int* hyp_px, int* inl_out, int* final_out, float* energy_out) {
  const Cam k{fx, fy, px, py};
  // getEye / pxToEye: float arithmetic, holes (depth 0) at the origin
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const int p = y * W + x;
      const unsigned short d = depth[p];
      float* e = eye_out + (size_t)p * 3;
      if (d == 0) {
        e[0] = e[1] = e[2] = 0.f;
      } else {
        e[0] = ((float)x - px) * (float)d / fx / depth_factor;
        e[1] = ((float)y - py) * (float)d / fy / depth_factor;
        e[2] = (float)d / depth_factor;
      }
    }
  auto eye_at = [&](int p) { return F3{eye_out[(size_t)p * 3], eye_out[(size_t)p * 3 + 1], eye_out[(size_t)p * 3 + 2]}; };
  std::vector<std::vector<int>> labels(C);
  for (int x = 0; x < W; x++)
    for (int y = 0; y < H; y++) labels[label[y * W + x]].push_back(y * W + x);
  std::vector<int> objs;
  for (int c = 1; c < C; c++)
    if ((float)labels[c].size() > 400.0f) objs.push_back(c);
  for (int i = 0; i < n_hyp * 13; i++) hyps_out[i] = 0;
  for (int i = 0; i < n_hyp; i++) hyps_out[i * 13] = -1;
  for (int i = 0; i < n_hyp * 3; i++) hyp_px[i] = -1;
  for (int i = 0; i < n_hyp * 8; i++) inl_out[i] = -1;
  for (int i = 0; i < C * 3; i++) final_out[i] = -1;
  for (int i = 0; i < C; i++) energy_out[i] = 0.f;
  for (int i = 0; i < 12 * C; i++) poses_out[i] = 0.f;
  if (objs.empty()) return 0;
  std::vector<std::vector<Hyp3>> hypmap(C);
  for (int h = 0; h < n_hyp; h++) {
    for (int it = 0; it < max_iter; it++) {
      TStream rs(seed, (uint32_t)h, kTagP3D, (uint32_t)it);
      const int obj = objs[rs.uniform((int)objs.size())];
      const auto& L = labels[obj];
      F3 E[3], O[3];
      int px3[3], n = 0;
      bool ok = true;
      for (int s = 0; s < 3 && ok; s++) {  // samplePoint3D x 3
        const int idx = L[rs.uniform((int)L.size())];
        const F3 eye = eye_at(idx);
        if (eye.z == 0) { ok = false; break; }
        double md = -1;
        for (int q = 0; q < n; q++) md = md < 0 ? norm3f(E[q], eye) : std::min(md, norm3f(E[q], eye));
        if (md > 0 && md < 0.01) { ok = false; break; }
        const F3 o = mode3d(vertmap, extents, C, obj, idx);
        if (o.x == 0 && o.y == 0 && o.z == 0) { ok = false; break; }
        md = -1;
        for (int q = 0; q < n; q++) md = md < 0 ? norm3f(O[q], o) : std::min(md, norm3f(O[q], o));
        if (md > 0 && md < 0.01) { ok = false; break; }
        E[n] = eye;
        O[n] = o;
        px3[n] = idx;
        n++;
      }
      if (!ok) continue;
      V3 a[3], b[3];
      for (int q = 0; q < 3; q++) {
        a[q] = {O[q].x, O[q].y, O[q].z};
        b[q] = {E[q].x, E[q].y, E[q].z};
      }
      const Pose P = kabsch(a, b, 3);
      bool out = false;
      for (int q = 0; q < 3 && !out; q++) out = !(nrm(b[q] - xform(P, a[q])) < 0.01);  // :1853-1860
      if (out) continue;
      const float e0 = extents[obj * 3] * 0.5f, e1 = extents[obj * 3 + 1] * 0.5f, e2 = extents[obj * 3 + 2] * 0.5f;
      const F3 bb3[8] = {{e0, e1, e2}, {-e0, e1, e2}, {e0, -e1, e2}, {-e0, -e1, e2},
                         {e0, e1, -e2}, {-e0, e1, -e2}, {e0, -e1, -e2}, {-e0, -e1, -e2}};
      if ((float)bb_area(P, bb3, k, W, H) < 400.0f) continue;  // :1871-1875
      Hyp3 hy;
      hy.h = h;
      hy.obj = obj;
      hy.pose = P;
      hypmap[obj].push_back(hy);
      hyps_out[h * 13] = (float)obj;
      for (int i = 0; i < 9; i++) hyps_out[h * 13 + 1 + i] = (float)P.R[i];
      for (int i = 0; i < 3; i++) hyps_out[h * 13 + 10 + i] = (float)P.t[i];
      for (int i = 0; i < 3; i++) hyp_px[h * 3 + i] = px3[i];
      break;
    }
  }
  for (int c = 0; c < C; c++) {
    auto& hs = hypmap[c];
    if (hs.empty()) continue;
    const auto& L = labels[c];
    const int N = (int)L.size();
    for (int round = 1; round <= 8; round++) {
      const int maxPixels = 1000 * round;
      const float rate = maxPixels / (float)N;
      const double q = 1.0 - (double)rate;
      std::vector<int> sub;  // visited pixels (holes step to the next pixel without a draw)
      for (int i = 0, j = 0; i < N;) {
        if (eye_at(L[i]).z == 0) { i++; continue; }
        sub.push_back(L[i]);
        if (rate < 1) i += subset_gap(seed, c, round - 1, j++, q);
        else i++;
      }
      for (auto& hy : hs) {
        hy.corr.clear();
        for (int p : sub) {
          const F3 e = eye_at(p);
          const F3 o = mode3d(vertmap, extents, C, c, p);
          const V3 d = V3{e.x, e.y, e.z} - xform(hy.pose, V3{o.x, o.y, o.z});
          if (nrm(d) < 0.01) hy.corr.push_back(Corr{o, e});
        }
        hy.inliers = (int)hy.corr.size();
        inl_out[hy.h * 8 + round - 1] = hy.inliers;
      }
      if (hs.size() > 1) {
        std::stable_sort(hs.begin(), hs.end(), [](const Hyp3& a, const Hyp3& b) { return a.inliers > b.inliers; });
        hs.erase(hs.begin() + hs.size() / 2, hs.end());
      }
      for (auto& hy : hs) {  // updateHyp3D (:1347-1370)
        if (hy.corr.size() < 4) continue;
        hy.corr = filter3d(hy.corr, seed, hy.h, round - 1);
        hy.pose = kabsch_corr(hy.corr);
      }
    }
    Hyp3& w = hs[0];
    final_out[c * 3] = w.h;
    final_out[c * 3 + 1] = w.inliers;
    int nh = 0;
    for (int h = 0; h < n_hyp; h++) nh += hyps_out[h * 13] == (float)c;
    final_out[c * 3 + 2] = nh;
    Pose P = w.pose;
    if (w.inliers > 10) {  // :1939-1944
      const std::vector<Corr> v = filter3d(w.corr, seed, w.h, 8);
      double x0[6], lb[6], ub[6], xb[6], fb;
      rod_m2v(P.R, x0);
      for (int i = 0; i < 3; i++) x0[3 + i] = P.t[i];
      const double rng[6] = {10 * 3.1415926 / 180, 10 * 3.1415926 / 180, 10 * 3.1415926 / 180, 0.1, 0.1, 0.5};
      for (int i = 0; i < 6; i++) {
        lb[i] = x0[i] - rng[i];
        ub[i] = x0[i] + rng[i];
      }
      nelder_mead([&](const double* x) { return energy3d(x, v); }, 6, x0, lb, ub, nm_evals, xb, &fb);
      rod_v2m(xb, P.R);
      for (int i = 0; i < 3; i++) P.t[i] = xb[3 + i];
      energy_out[c] = (float)fb;
    }
    for (int y = 0; y < 3; y++)
      for (int x = 0; x < 4; x++) poses_out[c + C * (y * 4 + x)] = x < 3 ? (float)P.R[y * 3 + x] : (float)P.t[y];
  }
  return (int)objs.size();
}
