// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// CPU restatement of the test-time pose refinement's numerical core
// (SURVEY.md §8(f) row 4): the projective point-to-plane ICP of
// lib/kinect_fusion (df::icp, src/optimization/icp.cpp:20-106 and the per-pixel
// kernel src/optimization/icp.cu:22-137, the linear system of
// include/df/optimization/linearSystems.h), the masked depth back-projection of
// Synthesizer::solveICP (lib/synthesize/synthesize.cpp:2140-2160 +
// df::backproject, src/image/backprojection.cu:10-27 with the Poly3 camera of
// include/df/camera/poly3.h at zero distortion), the translation re-centring
// (synthesize.cpp:2163-2233) and the pose energy of optEnergy
// (synthesize.cpp:2474-2526).
//
// Third-party arithmetic restated in closed form (absent here, unpinned):
// Sophus 1.x SE3<float> (exp with the SO3 expAndTheta small-angle branch at
// epsilon 1e-5, products with the 2 / (1 + |q|^2) renormalisation, point
// action through Eigen's Quaternion::_transformVector) and Eigen 3.3's
// LDLT<Upper> (diagonal pivoting, pseudo-inverse of zero pivots).  The
// reduction of the per-pixel systems (thrust::transform_reduce in float, order
// unspecified) is accumulated here in double in raster order: the oracle is
// the accurate member of that family, the HIP kernel's fixed-order float tree
// is checked against it with a tolerance.
#include "orc_common.h"
#include <cstring>
#include <vector>

namespace {

struct Quat { float w, x, y, z; };
struct SE3 { Quat q; float t[3]; };

// Eigen Quaternion::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
void rotate(const Quat& q, const float v[3], float o[3]) {
  float uv0 = q.y * v[2] - q.z * v[1];
  float uv1 = q.z * v[0] - q.x * v[2];
  float uv2 = q.x * v[1] - q.y * v[0];
  uv0 = uv0 + uv0; uv1 = uv1 + uv1; uv2 = uv2 + uv2;
  const float c0 = q.y * uv2 - q.z * uv1;
  const float c1 = q.z * uv0 - q.x * uv2;
  const float c2 = q.x * uv1 - q.y * uv0;
  o[0] = v[0] + q.w * uv0 + c0;
  o[1] = v[1] + q.w * uv1 + c1;
  o[2] = v[2] + q.w * uv2 + c2;
}

void act(const SE3& T, const float p[3], float o[3]) {
  rotate(T.q, p, o);
  o[0] = o[0] + T.t[0];
  o[1] = o[1] + T.t[1];
  o[2] = o[2] + T.t[2];
}

// Eigen quaternion product a * b
Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

// Sophus SE3 a * b: t = a.t + a.R b.t, q = a.q b.q renormalised by
// 2 / (1 + |q|^2) when |q|^2 != 1 (SO3Base::operator*=)
SE3 se3_mul(const SE3& a, const SE3& b) {
  SE3 r;
  float rt[3];
  rotate(a.q, b.t, rt);
  r.t[0] = a.t[0] + rt[0];
  r.t[1] = a.t[1] + rt[1];
  r.t[2] = a.t[2] + rt[2];
  r.q = qmul(a.q, b.q);
  const float n2 = r.q.w * r.q.w + r.q.x * r.q.x + r.q.y * r.q.y + r.q.z * r.q.z;
  if (n2 != 1.0f) {
    const float s = 2.0f / (1.0f + n2);
    r.q.w *= s; r.q.x *= s; r.q.y *= s; r.q.z *= s;
  }
  return r;
}

// Sophus SE3::exp of (upsilon, omega) (float, epsilon 1e-5)
SE3 se3_exp(const float a[6]) {
  const float w0 = a[3], w1 = a[4], w2 = a[5];
  const float theta_sq = w0 * w0 + w1 * w1 + w2 * w2;
  const float theta = std::sqrt(theta_sq);
  const float half_theta = 0.5f * theta;
  float imag, real;
  const float eps = 1e-5f;
  if (theta < eps) {
    const float theta_po4 = theta_sq * theta_sq;
    imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * theta_po4;
    real = 1.0f - 0.5f * theta_sq + (float)(1.0 / 384.0) * theta_po4;
  } else {
    imag = std::sin(half_theta) / theta;
    real = std::cos(half_theta);
  }
  SE3 r;
  r.q = {real, imag * w0, imag * w1, imag * w2};
  // Omega = hat(omega), V = I + (1 - cos) / theta^2 Omega + (theta - sin) / theta^3 Omega^2
  const float O[9] = {0.f, -w2, w1, w2, 0.f, -w0, -w1, w0, 0.f};
  float V[9];
  if (theta < eps) {  // V = so3.matrix()
    const Quat& q = r.q;
    const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z;
    const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    const float R[9] = {1.f - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.f - (txx + tzz), tyz - twx,
                        txz - twy, tyz + twx, 1.f - (txx + tyy)};
    std::memcpy(V, R, sizeof(V));
  } else {
    float O2[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) O2[i * 3 + j] = O[i * 3 + 0] * O[0 * 3 + j] + O[i * 3 + 1] * O[1 * 3 + j] + O[i * 3 + 2] * O[2 * 3 + j];
    const float c1 = (1.0f - std::cos(theta)) / theta_sq;
    const float c2 = (theta - std::sin(theta)) / (theta_sq * theta);
    for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.f : 0.f) + c1 * O[i] + c2 * O2[i];
  }
  for (int i = 0; i < 3; i++) r.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
  return r;
}

// Eigen 3.3 LDLT of the symmetric 6x6 A (upper triangle given, full matrix
// used) and solve A x = b.  Diagonal pivoting, zero pivots -> 0 in D^-1.
void ldlt_solve6(const float Ain[36], const float b[6], float x[6]) {
  float m[36];
  std::memcpy(m, Ain, sizeof(m));
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < i; j++) m[i * 6 + j] = m[j * 6 + i];  // lower from upper
  int tr[6];
  float temp[6];
  bool zero_all = false;
  for (int k = 0; k < 6; k++) {
    int big = k;
    float bv = std::fabs(m[k * 6 + k]);
    for (int i = k + 1; i < 6; i++)
      if (std::fabs(m[i * 6 + i]) > bv) { bv = std::fabs(m[i * 6 + i]); big = i; }
    tr[k] = big;
    if (big != k) {
      for (int j = 0; j < k; j++) std::swap(m[k * 6 + j], m[big * 6 + j]);
      for (int i = big + 1; i < 6; i++) std::swap(m[i * 6 + k], m[i * 6 + big]);
      std::swap(m[k * 6 + k], m[big * 6 + big]);
      for (int i = k + 1; i < big; i++) {
        const float t = m[i * 6 + k];
        m[i * 6 + k] = m[big * 6 + i];
        m[big * 6 + i] = t;
      }
    }
    const int rs = 5 - k;
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = m[j * 6 + j] * m[k * 6 + j];
      float s = 0.f;
      for (int j = 0; j < k; j++) s = s + m[k * 6 + j] * temp[j];
      m[k * 6 + k] -= s;
      for (int i = k + 1; i < 6; i++) {
        float si = 0.f;
        for (int j = 0; j < k; j++) si = si + m[i * 6 + j] * temp[j];
        m[i * 6 + k] -= si;
      }
    }
    const float akk = m[k * 6 + k];
    const bool valid = std::fabs(akk) > 0.f;
    if (k == 0 && !valid) {
      zero_all = true;
      break;
    }
    if (rs > 0 && valid)
      for (int i = k + 1; i < 6; i++) m[i * 6 + k] /= akk;
  }
  if (zero_all) {
    for (int i = 0; i < 6; i++) x[i] = 0.f;
    return;
  }
  for (int i = 0; i < 6; i++) x[i] = b[i];
  for (int k = 0; k < 6; k++) std::swap(x[k], x[tr[k]]);           // P b
  for (int i = 0; i < 6; i++)                                       // L^-1
    for (int j = 0; j < i; j++) x[i] -= m[i * 6 + j] * x[j];
  for (int i = 0; i < 6; i++) {                                     // D^+
    const float d = m[i * 6 + i];
    x[i] = std::fabs(d) > FLT_MIN ? x[i] / d : 0.f;
  }
  for (int i = 5; i >= 0; i--)                                      // L^-T
    for (int j = i + 1; j < 6; j++) x[i] -= m[j * 6 + i] * x[j];
  for (int k = 5; k >= 0; k--) std::swap(x[k], x[tr[k]]);          // P^T
}

// One icpKernel pixel (icp.cu:44-130): false when the pixel contributes a
// zero row; else J (1x6) and r.
bool icp_pixel(int x, int y, int W, int H, const float* live, const float* pv, const float* pn, float fx, float fy,
               float ppx, float ppy, float znear, float zfar, float max_error, const SE3& T, float J[6], float& r) {
  const float* v4 = pv + ((size_t)y * W + x) * 4;
  const float pd = v4[2];
  if (pd < znear || pd > zfar) return false;  // a NaN depth passes here and fails the border test
  float p[3];
  act(T, v4, p);
  const float qx = (p[0] / p[2]) * fx + ppx, qy = (p[1] / p[2]) * fy + ppy;
  const int u = orc::f2i_sat(qx + 0.5f), v = orc::f2i_sat(qy + 0.5f);  // GPU cvt: NaN -> 0
  const float border = 2.f;
  if ((float)u <= border || (float)u >= (float)(W - 1) - border || (float)v <= border ||
      (float)v >= (float)(H - 1) - border)
    return false;
  const float* lv = live + ((size_t)v * W + u) * 3;
  const float ld = lv[2];
  if (ld < znear || ld > zfar) return false;
  const float nrm = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  const float ray[3] = {p[0] / nrm, p[1] / nrm, p[2] / nrm};
  const float* n = pn + ((size_t)y * W + x) * 4;
  if (-(ray[0] * n[0] + ray[1] * n[1] + ray[2] * n[2]) < 0.1f) return false;
  const float e = n[0] * (lv[0] - p[0]) + n[1] * (lv[1] - p[1]) + n[2] * (lv[2] - p[2]);
  if (std::fabs(e) > max_error) return false;
  const float w = 1.0f / ld;
  // n^T [I | -hat(p)] : (n, p x n)
  J[0] = w * n[0];
  J[1] = w * n[1];
  J[2] = w * n[2];
  J[3] = w * (n[2] * p[1] - n[1] * p[2]);
  J[4] = w * (n[0] * p[2] - n[2] * p[0]);
  J[5] = w * (n[1] * p[0] - n[0] * p[1]);
  r = w * e;
  return true;
}

}  // namespace

// Masked depth -> live vertex map of one object (synthesize.cpp:2140-2160,
// backprojection.cu:10-27): d = depth / factor on label == obj, else 0;
// vertex = ((x - px) / fx d, (y - py) / fy d, d).
ORC_API void orc_icp_live_vertices(const uint16_t* depth, const int32_t* label, int H, int W, int obj, float factor,
                                   float fx, float fy, float px, float py, float* out) {
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const size_t j = (size_t)y * W + x;
      const float d = label[j] == obj ? (float)depth[j] / factor : 0.f;
      out[j * 3 + 0] = (((float)x - px) / fx) * d;
      out[j * 3 + 1] = (((float)y - py) / fy) * d;
      out[j * 3 + 2] = d;
    }
}

// df::icp (icp.cpp:20-106): `iterations` Gauss-Newton steps from the identity;
// each solves JTJ x = JTr (LDLT) and left-multiplies exp(x) into the
// accumulated update.  update = (qw, qx, qy, qz, tx, ty, tz); systems (optional)
// = per iteration the 21 upper-triangle JTJ entries (row-major) + 6 JTr + the
// contributing pixel count.
ORC_API void orc_icp(const float* live, const float* pv, const float* pn, int H, int W, float fx, float fy, float px,
                     float py, float znear, float zfar, float max_error, int iterations, float* update,
                     float* systems) {
  SE3 acc;
  acc.q = {1.f, 0.f, 0.f, 0.f};
  acc.t[0] = acc.t[1] = acc.t[2] = 0.f;
  for (int it = 0; it < iterations; it++) {
    double jtj[21] = {0}, jtr[6] = {0};
    int cnt = 0;
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        float J[6], r;
        if (!icp_pixel(x, y, W, H, live, pv, pn, fx, fy, px, py, znear, zfar, max_error, acc, J, r)) continue;
        cnt++;
        int k = 0;
        for (int i = 0; i < 6; i++)
          for (int j = i; j < 6; j++) jtj[k++] += (double)(J[i] * J[j]);
        for (int i = 0; i < 6; i++) jtr[i] += (double)(J[i] * r);
      }
    float A[36] = {0}, b[6], sol[6];
    int k = 0;
    for (int i = 0; i < 6; i++)
      for (int j = i; j < 6; j++) A[i * 6 + j] = (float)jtj[k++];
    for (int i = 0; i < 6; i++) b[i] = (float)jtr[i];
    if (systems) {
      for (int i = 0; i < 21; i++) systems[it * 28 + i] = (float)jtj[i];
      for (int i = 0; i < 6; i++) systems[it * 28 + 21 + i] = b[i];
      systems[it * 28 + 27] = (float)cnt;
    }
    ldlt_solve6(A, b, sol);
    acc = se3_mul(se3_exp(sol), acc);
  }
  update[0] = acc.q.w; update[1] = acc.q.x; update[2] = acc.q.y; update[3] = acc.q.z;
  update[4] = acc.t[0]; update[5] = acc.t[1]; update[6] = acc.t[2];
}

// Translation re-centring of solveICP (synthesize.cpp:2163-2205): over the
// object's pixels with depth > 0 and a non-NaN rendered vertmap, the mean of
// (live - model) over those with |n . (live - pred)| < max_error.  vx drops the
// class offset (vertmap.x - round(vertmap.x)).  out = (Tx, Ty, Tz, c).
ORC_API void orc_icp_center(const float* live, const int32_t* label, int obj, const float* vertmap, const float* pv,
                            const float* pn, int H, int W, float max_error, float* out) {
  double tx = 0, ty = 0, tz = 0;
  int c = 0;
  for (int j = 0; j < H * W; j++) {
    if (label[j] != obj || !(live[j * 3 + 2] > 0.f)) continue;
    const float vx = vertmap[j * 3 + 0] - std::round(vertmap[j * 3 + 0]);
    const float vy = vertmap[j * 3 + 1], vz = vertmap[j * 3 + 2];
    if (std::isnan(vx) || std::isnan(vy) || std::isnan(vz)) continue;
    const float* n = pn + (size_t)j * 4;
    const float* p = pv + (size_t)j * 4;
    const float* d = live + (size_t)j * 3;
    const float e = n[0] * (d[0] - p[0]) + n[1] * (d[1] - p[1]) + n[2] * (d[2] - p[2]);
    if (std::fabs(e) < max_error) {
      tx += (double)(d[0] - vx);
      ty += (double)(d[1] - vy);
      tz += (double)(d[2] - vz);
      c++;
    }
  }
  out[0] = c ? (float)(tx / c) : 0.f;
  out[1] = c ? (float)(ty / c) : 0.f;
  out[2] = c ? (float)(tz / c) : 0.f;
  out[3] = (float)c;
}

// optEnergy (synthesize.cpp:2474-2526) for K poses (qw qx qy qz tx ty tz; the
// quaternion normalised as the SE3 constructor does): mean over the object's
// pixels of |T p - v| where p (the rendered vertex) is not NaN and both depths
// lie strictly inside (znear, zfar).
ORC_API void orc_pose_energy(const float* live, const int32_t* label, int obj, const float* pv, int H, int W,
                             float znear, float zfar, const float* poses, int K, float* energy) {
  for (int k = 0; k < K; k++) {
    const float* P = poses + (size_t)k * 7;
    SE3 T;
    const float qn = std::sqrt(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
    T.q = {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
    T.t[0] = P[4]; T.t[1] = P[5]; T.t[2] = P[6];
    double dist = 0;
    int c = 0;
    for (int j = 0; j < H * W; j++) {
      if (label[j] != obj) continue;
      float p[3];
      act(T, pv + (size_t)j * 4, p);
      const float* v = live + (size_t)j * 3;
      if (!std::isnan(p[0]) && !std::isnan(p[1]) && !std::isnan(p[2]) && v[2] > znear && v[2] < zfar &&
          p[2] > znear && p[2] < zfar) {
        const float dx = p[0] - v[0], dy = p[1] - v[1], dz = p[2] - v[2];
        dist += (double)std::sqrt(dx * dx + dy * dy + dz * dz);
        c++;
      }
    }
    energy[k] = c ? (float)(dist / c) : 0.f;
  }
}

// SE3 helpers exposed for the host-side driver tests: c = a * b and exp(xi).
ORC_API void orc_se3_mul(const float* a, const float* b, float* c) {
  SE3 A, B;
  A.q = {a[0], a[1], a[2], a[3]}; A.t[0] = a[4]; A.t[1] = a[5]; A.t[2] = a[6];
  B.q = {b[0], b[1], b[2], b[3]}; B.t[0] = b[4]; B.t[1] = b[5]; B.t[2] = b[6];
  const SE3 C = se3_mul(A, B);
  c[0] = C.q.w; c[1] = C.q.x; c[2] = C.q.y; c[3] = C.q.z; c[4] = C.t[0]; c[5] = C.t[1]; c[6] = C.t[2];
}

ORC_API void orc_ldlt_solve6(const float* A, const float* b, float* x) { ldlt_solve6(A, b, x); }

// SegICP hypothesis score of solveICP (synthesize.cpp:2223-2330): model points
// (vertmap minus its class offset) and depth points (live vertices) of the
// object's pixels with depth > 0 and a finite vertmap, in raster order; per
// hypothesis each moved model point flags its nearest depth point within the
// radius (squared distance < radius^2, FLANN's test; ties -> lowest index);
// score = distinct flagged / model points; choose = first best (0 if none).
ORC_API void orc_icp_score(const float* live, const int32_t* label, int obj, const float* vertmap, int H, int W,
                           const float* hyps, int J, float radius, float* score, int32_t* choose) {
  std::vector<float> mp, dp;
  for (int j = 0; j < H * W; j++) {
    if (label[j] != obj || !(live[(size_t)j * 3 + 2] > 0.f)) continue;
    const float mx = vertmap[(size_t)j * 3 + 0] - std::round(vertmap[(size_t)j * 3 + 0]);
    const float my = vertmap[(size_t)j * 3 + 1], mz = vertmap[(size_t)j * 3 + 2];
    if (std::isnan(mx) || std::isnan(my) || std::isnan(mz)) continue;
    mp.insert(mp.end(), {mx, my, mz});
    dp.insert(dp.end(), {live[(size_t)j * 3 + 0], live[(size_t)j * 3 + 1], live[(size_t)j * 3 + 2]});
  }
  const int M = (int)(mp.size() / 3);
  const float r2 = radius * radius;
  float best_score = -FLT_MAX;
  int ch = -1;
  for (int h = 0; h < J; h++) {
    const float* P = hyps + (size_t)h * 7;
    SE3 T;
    const float qn = std::sqrt(P[0] * P[0] + P[1] * P[1] + P[2] * P[2] + P[3] * P[3]);
    T.q = {P[0] / qn, P[1] / qn, P[2] / qn, P[3] / qn};
    T.t[0] = P[4]; T.t[1] = P[5]; T.t[2] = P[6];
    std::vector<int> nn(M, -1);
#pragma omp parallel for schedule(static)
    for (int k = 0; k < M; k++) {
      float p[3];
      act(T, &mp[(size_t)k * 3], p);
      float best = r2;
      int bi = -1;
      for (int i = 0; i < M; i++) {
        const float dx = p[0] - dp[(size_t)i * 3], dy = p[1] - dp[(size_t)i * 3 + 1], dz = p[2] - dp[(size_t)i * 3 + 2];
        const float d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < best) { best = d2; bi = i; }
      }
      nn[k] = bi;
    }
    std::vector<char> flag(M, 0);
    int f = 0;
    for (int k = 0; k < M; k++)
      if (nn[k] >= 0 && !flag[nn[k]]) { flag[nn[k]] = 1; f++; }
    score[h] = M > 0 ? (float)f / (float)M : 0.f;
    if (score[h] > best_score) { best_score = score[h]; ch = h; }
  }
  *choose = M > 0 ? ch : 0;
}
