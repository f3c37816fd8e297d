// ORACLE — test infrastructure only.  CPU restatement of the class-aware
// greedy NMS of lib/utils/nms.py:3-32 (numpy, float32 rows) and of the pose
// combination of lib/fcn/test.py:197-211.
//
// Order: scores descending (nms.py:13 argsort()[::-1]); numpy leaves the order
// of equal scores unspecified (introsort / SIMD sort), so ties take the lower
// row index first — the canonical order the HIP kernel follows.  NaN scores
// sort last ascending in numpy, i.e. first here.  Arithmetic: float32 in the
// expression order of nms.py:11 and :17-25 (built with -ffp-contract=off).
#include "orc_common.h"
#include <algorithm>
#include <cmath>
#include <vector>

ORC_API int orc_box_nms(const float* dets, int R, int stride, float thresh, int* keep) {
  std::vector<int> order(R);
  for (int i = 0; i < R; i++) order[i] = i;
  auto score = [&](int i) { return dets[(size_t)i * stride + 6]; };
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    const float sa = score(a), sb = score(b);
    const bool na = std::isnan(sa), nb = std::isnan(sb);
    if (na || nb) return na && !nb;
    return sa > sb;
  });
  std::vector<float> area(R);
  for (int i = 0; i < R; i++) {
    const float* d = dets + (size_t)i * stride;
    area[i] = (d[4] - d[2] + 1.f) * (d[5] - d[3] + 1.f);  // nms.py:11
  }
  std::vector<char> removed(R, 0);
  int nk = 0;
  for (int a = 0; a < R; a++) {  // nms.py:15-30
    const int i = order[a];
    if (removed[a]) continue;
    keep[nk++] = i;
    const float* di = dets + (size_t)i * stride;
    for (int b = a + 1; b < R; b++) {
      if (removed[b]) continue;
      const int j = order[b];
      const float* dj = dets + (size_t)j * stride;
      const float xx1 = std::max(di[2], dj[2]), yy1 = std::max(di[3], dj[3]);
      const float xx2 = std::min(di[4], dj[4]), yy2 = std::min(di[5], dj[5]);
      const float w = std::max(0.f, xx2 - xx1 + 1.f), h = std::max(0.f, yy2 - yy1 + 1.f);
      const float inter = w * h;
      const float ovr = inter / (area[i] + area[j] - inter);
      if (ovr > thresh && dj[1] == di[1]) removed[b] = 1;  // nms.py:27
    }
  }
  return nk;
}

// test.py:199-211: rois[keep], poses_init[keep] with [:4] <- poses_pred[keep, 4cls:4cls+4]
ORC_API void orc_nms_combine(const float* rois, int stride, const float* poses_init, const float* poses_pred,
                             int pred_dim, const int* keep, int nk, float* rois_out, float* poses_out) {
  for (int q = 0; q < nk; q++) {
    const int i = keep[q];
    const int cls = (int)rois[(size_t)i * stride + 1];
    for (int c = 0; c < 7; c++) {
      rois_out[q * 7 + c] = rois[(size_t)i * stride + c];
      float v = poses_init[(size_t)i * 7 + c];
      if (c < 4 && cls >= 0 && poses_pred && 4 * cls + 3 < pred_dim) v = poses_pred[(size_t)i * pred_dim + 4 * cls + c];
      poses_out[q * 7 + c] = v;
    }
  }
}
