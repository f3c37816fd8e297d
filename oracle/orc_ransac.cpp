// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// CPU BASELINE: restatement of the reference CPU op `Houghvoting`
// (lib/hough_voting_layer/hough_voting_op.cc:104-231 Compute, :287-308 getLabels,
// :408-448 countInliers2D, :451-480 compute_width_height, :483-513 updateHyp2D /
// filterInliers2D, :516-857 estimateCenter, :923-999 compute_target_weight;
// ransac.h:40-142 TransHyp; Hypothesis.cpp:96-118 calcCenter;
// thread_rand.cpp:40-98 per-thread mt19937 seeded 1305 + tid).
//
// This op is a different algorithm from Houghvotinggpu (raw vertmap[+2]
// distance, 6-column boxes, preemptive RANSAC): it is the TIMING baseline of
// bench.py, never a numerical oracle for the GPU op (SURVEY.md finding 3).
// OpenCV is absent, so cv::solve(DECOMP_SVD) is restated as the minimum-norm
// least-squares solve through the eigen-decomposition of the 2x2 normal matrix,
// cv::projectPoints with rvec = 0 as a pinhole projection, Rodrigues(0) = I.
// Deviations that remove reference UB: getLabels is serialised (the reference
// push_back()s from an omp parallel loop, :293-299), compute_distance stops at
// the stored inlier list (the reference reads past it after filterInliers2D).
#include "orc_common.h"
#include <vector>
#include <map>
#include <random>
#include <algorithm>
#include <omp.h>

namespace {

struct Pt { double x, y; };

struct Hyp {
  int objID;
  Pt center;
  int bbw = 0, bbh = 0;
  float width_ = 0, height_ = 0;
  std::vector<std::pair<Pt, Pt>> inlierPts2D;  // (object dir, pixel)
  int maxPixels = 0, effPixels = 0, inliers = 0, refSteps = 0;
  bool operator<(const Hyp& o) const { return (float)inliers > (float)o.inliers; }
};

// thread_rand.cpp:31-69
struct ThreadRand {
  std::vector<std::mt19937> gens;
  void init(unsigned seed = 1305) {
    int n = omp_get_max_threads();
    gens.clear();
    for (int i = 0; i < n; i++) gens.emplace_back(i + seed);
  }
  int irand(int incMin, int excMax) {  // irand(min, max exclusive)
    std::uniform_int_distribution<int> dist(incMin, excMax - 1);
    return dist(gens[omp_get_thread_num()]);
  }
};
ThreadRand g_rand;
bool g_rand_init = false;

// Hypothesis.cpp:96-118: solve [m n] c = m*a + n*b in the least-squares,
// minimum-norm sense (cv::solve DECOMP_SVD).
Pt calc_center(const std::vector<std::pair<Pt, Pt>>& pts) {
  double a11 = 0, a12 = 0, a22 = 0, b1 = 0, b2 = 0;
  for (const auto& pr : pts) {
    double m1 = -pr.first.y, n1 = pr.first.x, a = pr.second.x, b = pr.second.y;
    double rhs = m1 * a + n1 * b;
    a11 += m1 * m1; a12 += m1 * n1; a22 += n1 * n1;
    b1 += m1 * rhs; b2 += n1 * rhs;
  }
  // eigen-decomposition of the symmetric [[a11 a12][a12 a22]]
  double tr = a11 + a22, det = a11 * a22 - a12 * a12;
  double disc = std::sqrt(std::max(0.0, tr * tr / 4 - det));
  double l1 = tr / 2 + disc, l2 = tr / 2 - disc;
  double v1x, v1y;
  if (std::fabs(a12) > 1e-300) { v1x = l1 - a22; v1y = a12; }
  else if (a11 >= a22) { v1x = 1; v1y = 0; }
  else { v1x = 0; v1y = 1; }
  double nv = std::sqrt(v1x * v1x + v1y * v1y);
  v1x /= nv; v1y /= nv;
  double v2x = -v1y, v2y = v1x;
  double eps = 1e-12 * std::max(std::fabs(l1), 1e-300);  // SVD rank threshold on sigma^2
  double cx = 0, cy = 0;
  double p1 = v1x * b1 + v1y * b2, p2 = v2x * b1 + v2y * b2;
  if (l1 > eps) { cx += v1x * p1 / l1; cy += v1y * p1 / l1; }
  if (l2 > eps) { cx += v2x * p2 / l2; cy += v2y * p2 / l2; }
  return {cx, cy};
}

inline float point2line(Pt x, Pt n, Pt p) {  // op.cc:392-403
  float n1 = (float)-n.y, n2 = (float)n.x, p1 = (float)p.x, p2 = (float)p.y, x1 = (float)x.x, x2 = (float)x.y;
  return fabsf(n1 * (x1 - p1) + n2 * (x2 - p2)) / sqrtf(n1 * n1 + n2 * n2);
}
inline float angle_dist(Pt x, Pt n, Pt p) { return (float)(n.x * (x.x - p.x) + n.y * (x.y - p.y)); }  // op.cc:406

inline bool inlier(const Hyp& h, Pt obj, Pt pt, float thr) {
  float d = (float)std::sqrt((h.center.x - pt.x) * (h.center.x - pt.x) + (h.center.y - pt.y) * (h.center.y - pt.y));
  return point2line(h.center, obj, pt) < thr && angle_dist(h.center, obj, pt) > 0 && d < (float)std::max(h.bbw, h.bbh);
}

inline Pt mode2d(int obj, int index, const float* vert, int W, int C, float& dist) {  // op.cc:327-338
  size_t off = 3 * (size_t)obj + 3 * (size_t)C * (size_t)index;
  dist = vert[off + 2];
  return {vert[off], vert[off + 1]};
}

// op.cc:408-448
void count_inliers(Hyp& h, const float* vert, const std::vector<std::vector<int>>& labels, float thr, int W, int C,
                   int batch) {
  h.inlierPts2D.clear();
  h.inliers = 0;
  h.effPixels = 0;
  h.maxPixels += batch;
  const std::vector<int>& L = labels[h.objID];
  int maxPt = (int)L.size();
  float successRate = (float)h.maxPixels / (float)maxPt;
  std::mt19937 generator;
  std::negative_binomial_distribution<int> distribution(1, successRate < 1 ? successRate : 0.5f);
  for (unsigned ptIdx = 0; ptIdx < (unsigned)maxPt;) {
    int index = L[ptIdx];
    Pt pt{(double)(index % W), (double)(index / W)};
    h.effPixels++;
    float dist;
    Pt obj = mode2d(h.objID, index, vert, W, C, dist);
    if (inlier(h, obj, pt, thr)) {
      h.inlierPts2D.push_back({obj, pt});
      h.inliers++;
    }
    if (successRate < 1) ptIdx += std::max(1, distribution(generator));
    else ptIdx++;
  }
}

// op.cc:451-480
void compute_width_height(Hyp& h, const float* vert, const std::vector<std::vector<int>>& labels, float thr, int W,
                          int C) {
  float w = -1, hh = -1;
  for (int index : labels[h.objID]) {
    Pt pt{(double)(index % W), (double)(index / W)};
    float dist;
    Pt obj = mode2d(h.objID, index, vert, W, C, dist);
    if (inlier(h, obj, pt, thr)) {
      float x = (float)std::fabs(pt.x - h.center.x), y = (float)std::fabs(pt.y - h.center.y);
      if (x > w) w = x;
      if (y > hh) hh = y;
    }
  }
  h.width_ = 2 * w;
  h.height_ = 2 * hh;
}

void update_hyp(Hyp& h, int maxPixels) {  // op.cc:483-513
  if (h.inlierPts2D.size() < 4) return;
  if ((int)h.inlierPts2D.size() >= maxPixels) {
    std::vector<std::pair<Pt, Pt>> f;
    for (int i = 0; i < maxPixels; i++) f.push_back(h.inlierPts2D[g_rand.irand(0, (int)h.inlierPts2D.size())]);
    h.inlierPts2D = f;
  }
  h.center = calc_center(h.inlierPts2D);
}

std::vector<Hyp*> working_queue(std::map<int, std::vector<Hyp>>& m, int maxIt, int is_train) {  // op.cc:362-383
  std::vector<Hyp*> q;
  for (auto& kv : m)
    for (auto& h : kv.second)
      if (is_train ? h.refSteps < maxIt : ((int)kv.second.size() > 1 || h.refSteps < maxIt)) q.push_back(&h);
  return q;
}

// projected 2-D box extent of the class 3-D box at depth d (op.cc:634-656)
void bb_at_depth(const float* ext, double d, float fx, float fy, float px, float py, int& bw, int& bh) {
  float xh = (float)(ext[0] * 0.5), yh = (float)(ext[1] * 0.5), zh = (float)(ext[2] * 0.5);
  int minX = 10000000, maxX = -10000000, minY = 10000000, maxY = -10000000;
  for (int i = 0; i < 8; i++) {
    double X = (i & 1) ? -xh : xh, Y = (i & 2) ? -yh : yh, Z = ((i & 4) ? -zh : zh) + d;
    float x = (float)(fx * (X / Z) + px), y = (float)(fy * (Y / Z) + py);
    minX = (int)std::min((float)minX, x); minY = (int)std::min((float)minY, y);
    maxX = (int)std::max((float)maxX, x); maxY = (int)std::max((float)maxY, y);
  }
  bw = maxX - minX + 1;
  bh = maxY - minY + 1;
}

}  // namespace

// One image of estimateCenter (op.cc:516-857).  Output rows of 13 floats:
// [b, cls, x1, y1, x2, y2, qw, qx, qy, qz, tx, ty, tz]; returns the row count.
static int estimate_center(const int* labelmap, const float* vert, const float* extents, int batch, int H, int W,
                           int C, int is_train, float fx, float fy, float px, float py, std::vector<float>& out) {
  const int maxIterations = 10000000;
  const float minArea = 400, minDist2D = 10, inlierThreshold = 0.5f;
  const int ransacIterations = 256, preemptiveBatch = 100, maxPixels = 1000, refIt = is_train ? 4 : 8;
  std::vector<std::vector<int>> labels(C);
  std::vector<int> object_ids;
  for (int x = 0; x < W; x++)  // column-major, serialised (op.cc:293-299)
    for (int y = 0; y < H; y++) {
      int l = labelmap[y * W + x];
      if (l >= 0 && l < C) labels[l].push_back(y * W + x);
    }
  for (int i = 1; i < C; i++)
    if ((float)labels[i].size() > minArea) object_ids.push_back(i);
  if (object_ids.empty()) return 0;
  std::map<int, std::vector<Hyp>> hypMap;
#pragma omp parallel for
  for (int h = 0; h < ransacIterations; h++)
    for (int it = 0; it < maxIterations; it++) {
      int objID = object_ids[g_rand.irand(0, (int)object_ids.size())];
      const std::vector<int>& L = labels[objID];
      int i1 = L[g_rand.irand(0, (int)L.size())];
      Pt pt1{(double)(i1 % W), (double)(i1 / W)};
      float d1, d2;
      Pt o1 = mode2d(objID, i1, vert, W, C, d1);
      if (d1 < 0) continue;
      int i2 = L[g_rand.irand(0, (int)L.size())];
      Pt pt2{(double)(i2 % W), (double)(i2 / W)};
      if (std::sqrt((pt1.x - pt2.x) * (pt1.x - pt2.x) + (pt1.y - pt2.y) * (pt1.y - pt2.y)) < minDist2D) continue;
      Pt o2 = mode2d(objID, i2, vert, W, C, d2);
      if (d2 < 0) continue;
      float distance = (d1 + d2) / 2.f;
      std::vector<std::pair<Pt, Pt>> pts{{o1, pt1}, {o2, pt2}};
      Pt center = calc_center(pts);
      int x = (int)center.x, y = (int)center.y;
      if (C > 2 && x >= 0 && x < W && y >= 0 && y < H && labelmap[y * W + x] == 0) continue;
      Hyp hyp;
      hyp.objID = objID;
      hyp.center = center;
      bb_at_depth(extents + 3 * objID, distance, fx, fy, px, py, hyp.bbw, hyp.bbh);
      double lim = std::max(hyp.bbw, hyp.bbh);
      double n1 = std::sqrt((pt1.x - (float)center.x) * (pt1.x - (float)center.x) + (pt1.y - (float)center.y) * (pt1.y - (float)center.y));
      double n2 = std::sqrt((pt2.x - (float)center.x) * (pt2.x - (float)center.x) + (pt2.y - (float)center.y) * (pt2.y - (float)center.y));
      if (n1 > lim || n2 > lim) continue;
#pragma omp critical
      hypMap[objID].push_back(hyp);
      break;
    }
  std::vector<int> objList;
  for (auto& kv : hypMap) objList.push_back(kv.first);
  std::vector<Hyp*> wq = working_queue(hypMap, refIt, is_train);
  while (!wq.empty()) {
#pragma omp parallel for
    for (int h = 0; h < (int)wq.size(); h++)
      count_inliers(*wq[h], vert, labels, inlierThreshold, W, C, preemptiveBatch);
    for (int objID : objList) {
      auto& v = hypMap[objID];
      if (v.size() > 1) {
        std::sort(v.begin(), v.end());
        v.erase(v.begin() + v.size() / 2, v.end());
      }
    }
    wq = working_queue(hypMap, refIt, is_train);
#pragma omp parallel for
    for (int h = 0; h < (int)wq.size(); h++) {
      update_hyp(*wq[h], maxPixels);
      wq[h]->refSteps++;
    }
    wq = working_queue(hypMap, refIt, is_train);
  }
  std::vector<Hyp*> all;
  for (auto& kv : hypMap)
    for (auto& h : kv.second) all.push_back(&h);
  std::vector<std::vector<float>> rows(all.size());
#pragma omp parallel for
  for (int k = 0; k < (int)all.size(); k++) {
    Hyp& h = *all[k];
    float rx = (float)((h.center.x - px) / fx), ry = (float)((h.center.y - py) / fy);
    float distance = 0;  // TransHyp::compute_distance (ransac.h:108-119)
    int n = std::min<int>(h.inliers, (int)h.inlierPts2D.size());
    for (int i = 0; i < n; i++) {
      int xx = (int)h.inlierPts2D[i].second.x, yy = (int)h.inlierPts2D[i].second.y;
      distance += vert[3 * (size_t)h.objID + 3 * (size_t)C * ((size_t)yy * W + xx) + 2];
    }
    distance /= (float)h.inliers;
    compute_width_height(h, vert, labels, inlierThreshold, W, C);
    float scale = 0.05f;
    std::vector<float> r(13);
    r[0] = (float)batch;
    r[1] = (float)h.objID;
    r[2] = (float)(h.center.x - h.width_ * (0.5 + scale));
    r[3] = (float)(h.center.y - h.height_ * (0.5 + scale));
    r[4] = (float)(h.center.x + h.width_ * (0.5 + scale));
    r[5] = (float)(h.center.y + h.height_ * (0.5 + scale));
    r[6] = 1; r[7] = 0; r[8] = 0; r[9] = 0;  // Rodrigues(0) -> identity quaternion
    r[10] = rx * distance; r[11] = ry * distance; r[12] = distance;
    if (is_train) {
      float x1 = r[2], y1 = r[3], x2 = r[4], y2 = r[5], ww = x2 - x1, hh = y2 - y1;
      const int jit[8][2] = {{-1, -1}, {1, -1}, {-1, 1}, {1, 1}, {0, -1}, {-1, 0}, {0, 1}, {1, 0}};
      std::vector<float> base = r;
      for (int j = 0; j < 8; j++) {
        std::vector<float> q = base;
        q[2] = (float)(x1 + jit[j][0] * 0.05 * ww);
        q[3] = (float)(y1 + jit[j][1] * 0.05 * hh);
        q[4] = q[2] + ww;
        q[5] = q[3] + hh;
        r.insert(r.end(), q.begin(), q.end());
      }
    }
    rows[k] = r;
  }
  int cnt = 0;
  for (auto& r : rows) { out.insert(out.end(), r.begin(), r.end()); cnt += (int)r.size() / 13; }
  return cnt;
}

// Batch driver (op.cc:104-231).  rows_out capacity `cap` rows of 13 floats.
// Returns the number of rows (excluding the reference's dummy row).
ORC_API int orc_ransac_hough(const int* label, const float* vertex, const float* extents, const float* meta,
                             int num_meta, int B, int H, int W, int C, int is_train, int num_threads,
                             float* rows_out, int cap) {
  if (num_threads > 0) omp_set_num_threads(num_threads);
  if (!g_rand_init || (int)g_rand.gens.size() != omp_get_max_threads()) { g_rand.init(); g_rand_init = true; }
  std::vector<float> out;
  int total = 0;
  for (int n = 0; n < B; n++) {
    const float* m = meta + (size_t)n * num_meta;
    total += estimate_center(label + (size_t)n * H * W, vertex + (size_t)n * H * W * 3 * C, extents, n, H, W, C,
                             is_train, m[0], m[4], m[2], m[5], out);
  }
  int k = std::min(total, cap);
  std::copy(out.begin(), out.begin() + (size_t)k * 13, rows_out);
  return total;
}
