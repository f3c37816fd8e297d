// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// Restatement of the reference `Averagedistance` op (ADD / ADD-S pose loss) as
// the GPU kernels define it — the CPU twin (average_distance_loss_op.cc:71-219)
// ignores symmetry, so lib/average_distance_loss/average_distance_loss_op_gpu.cu.cc
// is the spec:
//   AveragedistanceForward   cu.cc:34-206  (per (row, point))
//   sum_losses_gradients     cu.cc:209-252 (sequential sums over points)
//   thrust::reduce           cu.cc:333-334 (here: sequential over rows)
//   AveragedistanceBackward  cu.cc:346-354
#include "orc_common.h"
#include <vector>

namespace {
// cu.cc:63-71 / :82-90 (quaternion (s,u,v,w) -> rotation, unnormalised)
inline void quat2rot(float s, float u, float v, float w, float* r) {
  r[0] = s * s + u * u - v * v - w * w;
  r[1] = 2 * (u * v - s * w);
  r[2] = 2 * (u * w + s * v);
  r[3] = 2 * (u * v + s * w);
  r[4] = s * s - u * u + v * v - w * w;
  r[5] = 2 * (v * w - s * u);
  r[6] = 2 * (u * w - s * v);
  r[7] = 2 * (v * w + s * u);
  r[8] = s * s - u * u - v * v + w * w;
}
}  // namespace

// pred/target/weight: (R, 4C); points: (C, P, 3); symmetry: (C).
// loss_out: scalar; diff_out: (R, 4C) = bottom_diff; row_loss_out (R) optional.
ORC_API void orc_add_loss_fwd(const float* pred, const float* target, const float* weight, const float* points,
                              const float* symmetry, int R, int C, int P, float margin, float* loss_out,
                              float* diff_out, float* row_loss_out) {
  const int PC = 4 * C;
  std::vector<float> losses((size_t)P), diffs((size_t)P * 4);
  float total = 0.f;
  for (int n = 0; n < R; n++) {
    int index_cls = -1;
    float rot[54];
    float s = 0, u = 0, v = 0, w = 0;
    for (int i = 0; i < PC; i += 4) {  // cu.cc:48-92
      int index = n * PC + i;
      if (weight[index] > 0) {
        index_cls = i / 4;
        quat2rot(target[index + 0], target[index + 1], target[index + 2], target[index + 3], rot);
        s = pred[index + 0]; u = pred[index + 1]; v = pred[index + 2]; w = pred[index + 3];
        quat2rot(s, u, v, w, rot + 9);
        break;
      }
    }
    for (int c = 0; c < PC; c++) diff_out[(size_t)n * PC + c] = 0.f;
    if (index_cls == -1) {
      if (row_loss_out) row_loss_out[n] = 0.f;
      continue;
    }
    // derivative matrices (cu.cc:97-139), functions of the predicted quaternion
    float* d0 = rot + 18; float* d1 = rot + 27; float* d2 = rot + 36; float* d3 = rot + 45;
    const float a0[9] = {2 * s, -2 * w, 2 * v, 2 * w, 2 * s, -2 * u, -2 * v, 2 * u, 2 * s};
    const float a1[9] = {2 * u, 2 * v, 2 * w, 2 * v, -2 * u, -2 * s, 2 * w, 2 * s, -2 * u};
    const float a2[9] = {-2 * v, 2 * u, 2 * s, 2 * u, 2 * v, 2 * w, -2 * s, 2 * w, -2 * v};
    const float a3[9] = {-2 * w, -2 * s, 2 * u, 2 * s, -2 * w, 2 * v, 2 * u, 2 * v, 2 * w};
    for (int k = 0; k < 9; k++) { d0[k] = a0[k]; d1[k] = a1[k]; d2[k] = a2[k]; d3[k] = a3[k]; }
    const float* pts = points + (size_t)index_cls * P * 3;
    const float* Rg = rot;
    const float* Rp = rot + 9;
    for (int p = 0; p < P; p++) {
      losses[p] = 0.f;
      float* dd = &diffs[(size_t)p * 4];
      dd[0] = dd[1] = dd[2] = dd[3] = 0.f;
      const float* X = pts + (size_t)p * 3;
      float x1 = Rp[0] * X[0] + Rp[1] * X[1] + Rp[2] * X[2];
      float y1 = Rp[3] * X[0] + Rp[4] * X[1] + Rp[5] * X[2];
      float z1 = Rp[6] * X[0] + Rp[7] * X[1] + Rp[8] * X[2];
      const float* Xm = X;
      if (symmetry[index_cls] > 0) {  // cu.cc:150-172
        float dmin = FLT_MAX;
        for (int i = 0; i < P; i++) {
          const float* Y = pts + (size_t)i * 3;
          float x2 = Rg[0] * Y[0] + Rg[1] * Y[1] + Rg[2] * Y[2];
          float y2 = Rg[3] * Y[0] + Rg[4] * Y[1] + Rg[5] * Y[2];
          float z2 = Rg[6] * Y[0] + Rg[7] * Y[1] + Rg[8] * Y[2];
          float distance = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2);
          if (distance < dmin) { dmin = distance; Xm = Y; }
        }
      }
      float x2 = Rg[0] * Xm[0] + Rg[1] * Xm[1] + Rg[2] * Xm[2];
      float y2 = Rg[3] * Xm[0] + Rg[4] * Xm[1] + Rg[5] * Xm[2];
      float z2 = Rg[6] * Xm[0] + Rg[7] * Xm[1] + Rg[8] * Xm[2];
      float distance = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2);
      if (distance < margin) continue;  // cu.cc:178-179
      losses[p] = (float)((double)(distance - margin) / (2.0 * R * P));  // cu.cc:181
      const float bn = (float)(R * P);
      for (int j = 0; j < 3; j++) {  // cu.cc:183-203
        float diff = j == 0 ? x1 - x2 : (j == 1 ? y1 - y2 : z1 - z2);
        for (int k = 0; k < 3; k++) {
          dd[0] += diff * X[k] * d0[j * 3 + k] / bn;
          dd[1] += diff * X[k] * d1[j * 3 + k] / bn;
          dd[2] += diff * X[k] * d2[j * 3 + k] / bn;
          dd[3] += diff * X[k] * d3[j * 3 + k] / bn;
        }
      }
    }
    // sum_losses_gradients (cu.cc:236-250): sequential over points
    float lb = 0.f;
    for (int p = 0; p < P; p++) lb += losses[p];
    for (int q = 0; q < 4; q++) {
      float acc = 0.f;
      for (int p = 0; p < P; p++) acc += diffs[(size_t)p * 4 + q];
      diff_out[(size_t)n * PC + 4 * index_cls + q] = acc;
    }
    if (row_loss_out) row_loss_out[n] = lb;
    total += lb;
  }
  *loss_out = total;
}

// cu.cc:346-354
ORC_API void orc_add_loss_bwd(const float* top_diff, const float* bottom_diff, int n, float* out) {
  for (int i = 0; i < n; i++) out[i] = top_diff[0] * bottom_diff[i];
}
