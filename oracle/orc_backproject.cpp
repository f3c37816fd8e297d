// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// Restatement of the reference `Backproject` / `BackprojectGrad` ops.
//  forward : backprojecting_op.cc:164-251 (CPU kernel; identical arithmetic to
//            BackprojectForward, backprojecting_op_gpu.cu.cc:16-126, minus the
//            GPU kernel's per-channel label write race)
//  backward: BackprojectBackward (backprojecting_op_gpu.cu.cc:158-217)
// meta layout (hough_voting_gpu_op.cc:341-347): K[0..8] Kinv[9..17]
// world2live[18..29] live2world[30..41] voxel step[42..44] voxel min[45..47].
#include "orc_common.h"
#include <algorithm>

// data (B,H,W,Ch) label (B,H,W,NC) depth (B,H,W) meta (B,num_meta) label3d (B,G,G,G,NC)
// -> top_data (B,G,G,G,Ch), top_label (B,G,G,G,NC), top_flag (B,G,G,G,Ch)
ORC_API void orc_backproject_fwd(const float* data, const float* label, const float* depth, const float* meta_all,
                                 int num_meta, const float* label3d, int B, int H, int W, int Ch, int NC, int G,
                                 int ks, float threshold, float* top_data, float* top_label, float* top_flag) {
  for (int n = 0; n < B; n++) {
    const float* m = meta_all + (size_t)n * num_meta;
    for (int d = 0; d < G; d++)
      for (int h = 0; h < G; h++)
        for (int w = 0; w < G; w++) {
          float X = (float)d * m[42] + m[45];
          float Y = (float)h * m[43] + m[46];
          float Z = (float)w * m[44] + m[47];
          float X1 = m[18] * X + m[19] * Y + m[20] * Z + m[21];
          float Y1 = m[22] * X + m[23] * Y + m[24] * Z + m[25];
          float Z1 = m[26] * X + m[27] * Y + m[28] * Z + m[29];
          float x1 = m[0] * X1 + m[1] * Y1 + m[2] * Z1;
          float x2 = m[3] * X1 + m[4] * Y1 + m[5] * Z1;
          float x3 = m[6] * X1 + m[7] * Y1 + m[8] * Z1;
          int px = orc::f2i_sat(roundf(x1 / x3));
          int py = orc::f2i_sat(roundf(x2 / x3));
          size_t vox = (((size_t)n * G + d) * G + h) * G + w;
          float* td = top_data + vox * Ch;
          float* tl = top_label + vox * NC;
          float* tf = top_flag + vox * Ch;
          for (int c = 0; c < Ch; c++) td[c] = 0.f;
          for (int c = 0; c < NC; c++) tl[c] = 0.f;
          int count = 0;
          // x outer, y inner (cc:199-200); 64-bit loop bounds avoid overflow at
          // saturated px/py
          for (long x = (long)px - ks; x <= (long)px + ks; x++)
            for (long y = (long)py - ks; y <= (long)py + ks; y++) {
              if (x >= 0 && x < W && y >= 0 && y < H) {
                size_t ip = ((size_t)n * H + y) * W + x;
                float dep = depth[ip];
                float dvoxel = Z1;
                if (fabsf(dep - dvoxel) < threshold) {
                  count++;
                  for (int c = 0; c < Ch; c++) td[c] += data[ip * Ch + c];
                  for (int c = 0; c < NC; c++) tl[c] += label[ip * NC + c];
                }
              }
            }
          if (count == 0) {
            for (int c = 0; c < Ch; c++) tf[c] = 0.f;
            for (int c = 0; c < NC; c++) tl[c] = label3d[vox * NC + c];
          } else {
            for (int c = 0; c < Ch; c++) { td[c] /= (float)count; tf[c] = 1.f; }
            for (int c = 0; c < NC; c++) tl[c] /= (float)count;
          }
        }
  }
}

// top_diff (B,G,G,G,Ch) -> bottom_diff (B,H,W,Ch)
ORC_API void orc_backproject_bwd(const float* top_diff, const float* depth, const float* meta_all, int num_meta,
                                 int B, int H, int W, int Ch, int G, float* bottom_diff) {
  for (int n = 0; n < B; n++) {
    const float* m = meta_all + (size_t)n * num_meta;
    for (int h = 0; h < H; h++)
      for (int w = 0; w < W; w++) {
        float dep = depth[((size_t)n * H + h) * W + w];
        float RX = m[9] * (float)w + m[10] * (float)h + m[11];
        float RY = m[12] * (float)w + m[13] * (float)h + m[14];
        float RZ = m[15] * (float)w + m[16] * (float)h + m[17];
        float X = dep * RX, Y = dep * RY, Z = dep * RZ;
        float X1 = m[30] * X + m[31] * Y + m[32] * Z + m[33];
        float Y1 = m[34] * X + m[35] * Y + m[36] * Z + m[37];
        float Z1 = m[38] * X + m[39] * Y + m[40] * Z + m[41];
        int vd = orc::f2i_sat(roundf((X1 - m[45]) / m[42]));
        int vh = orc::f2i_sat(roundf((Y1 - m[46]) / m[43]));
        int vw = orc::f2i_sat(roundf((Z1 - m[47]) / m[44]));
        float* bd = bottom_diff + (((size_t)n * H + h) * W + w) * Ch;
        if (vd >= 0 && vd < G && vh >= 0 && vh < G && vw >= 0 && vw < G) {
          const float* td = top_diff + ((((size_t)n * G + vd) * G + vh) * G + vw) * Ch;
          for (int c = 0; c < Ch; c++) bd[c] = td[c];
        } else {
          for (int c = 0; c < Ch; c++) bd[c] = 0.f;
        }
      }
  }
}
