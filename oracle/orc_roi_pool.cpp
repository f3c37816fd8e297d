// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// Restatement of the reference `RoiPool` / `RoiPoolGrad` ops on NHWC features.
//  forward : ROIPoolForward (lib/roi_pooling_layer/roi_pooling_op_gpu.cu.cc:19-101),
//            same semantics as the CPU kernel roi_pooling_op.cc:79-239
//  backward: ROIPoolBackward (roi_pooling_op_gpu.cu.cc:134-229)
#include "orc_common.h"
#include <vector>
#include <algorithm>

namespace {
struct RoiGeom { int b, cls, sw, sh, ew, eh; float bin_h, bin_w; };

// roi_pooling_op_gpu.cu.cc:45-59 (round = half away from zero, roundf)
inline RoiGeom roi_geom(const float* r, float scale, int ph_, int pw_) {
  RoiGeom g;
  g.b = orc::f2i_sat(r[0]);
  g.cls = orc::f2i_sat(r[1]);
  g.sw = orc::f2i_sat(roundf(r[2] * scale));
  g.sh = orc::f2i_sat(roundf(r[3] * scale));
  g.ew = orc::f2i_sat(roundf(r[4] * scale));
  g.eh = orc::f2i_sat(roundf(r[5] * scale));
  int roi_width = std::max(g.ew - g.sw + 1, 1);
  int roi_height = std::max(g.eh - g.sh + 1, 1);
  g.bin_h = (float)roi_height / (float)ph_;
  g.bin_w = (float)roi_width / (float)pw_;
  return g;
}
}  // namespace

// top: (R, PH, PW, Cout) with Cout = pool_channel ? 1 : C; argmax int32 same shape.
ORC_API int orc_roi_pool_fwd(const float* data, int B, int H, int W, int C, const float* rois, int R, int roi_stride,
                             float scale, int PH, int PW, int pool_channel, float* top, int* argmax) {
  const int Cout = pool_channel ? 1 : C;
  for (int n = 0; n < R; n++) {
    RoiGeom g = roi_geom(rois + (size_t)n * roi_stride, scale, PH, PW);
    if (g.b < 0 || g.b >= B) return -1;
    const float* bd = data + (size_t)g.b * H * W * C;
    for (int ph = 0; ph < PH; ph++)
      for (int pw = 0; pw < PW; pw++) {
        int hstart = (int)floorf((float)ph * g.bin_h);
        int wstart = (int)floorf((float)pw * g.bin_w);
        int hend = (int)ceilf((float)(ph + 1) * g.bin_h);
        int wend = (int)ceilf((float)(pw + 1) * g.bin_w);
        hstart = std::min(std::max(hstart + g.sh, 0), H);
        hend = std::min(std::max(hend + g.sh, 0), H);
        wstart = std::min(std::max(wstart + g.sw, 0), W);
        wend = std::min(std::max(wend + g.sw, 0), W);
        bool is_empty = (hend <= hstart) || (wend <= wstart);
        for (int c = 0; c < Cout; c++) {
          float maxval = is_empty ? 0.f : -FLT_MAX;
          int maxidx = -1;
          for (int h = hstart; h < hend; h++)
            for (int w = wstart; w < wend; w++) {
              int bi = pool_channel ? (h * W + w) * C + g.cls : (h * W + w) * C + c;
              if (bd[bi] > maxval) { maxval = bd[bi]; maxidx = bi; }
            }
          size_t o = (((size_t)n * PH + ph) * PW + pw) * Cout + c;
          top[o] = maxval;
          argmax[o] = maxidx;
        }
      }
  }
  return 0;
}

// bottom_diff: (B, H, W, C).  Loop order per bottom element = reference order
// (roi ascending, ph ascending, pw ascending); RoIs that the reference skips
// (batch mismatch, class mismatch for pool_channel, outside the RoI) add nothing.
ORC_API int orc_roi_pool_bwd(const float* top_diff, const int* argmax, int B, int H, int W, int C, const float* rois,
                             int R, int roi_stride, float scale, int PH, int PW, int pool_channel, float* bottom_diff) {
  const int Cout = pool_channel ? 1 : C;
  std::vector<RoiGeom> geo(R);
  for (int n = 0; n < R; n++) geo[n] = roi_geom(rois + (size_t)n * roi_stride, scale, PH, PW);
  // every bottom element is independent (its own ordered sum): rows in parallel
#pragma omp parallel for collapse(2) schedule(static)
  for (int n = 0; n < B; n++)
    for (int h = 0; h < H; h++)
      for (int w = 0; w < W; w++)
        for (int c = 0; c < C; c++) {
          float gradient = 0.f;
          for (int r = 0; r < R; r++) {
            const RoiGeom& g = geo[r];
            if (n != g.b) continue;
            if (pool_channel && c != g.cls) continue;
            if (!(w >= g.sw && w <= g.ew && h >= g.sh && h <= g.eh)) continue;
            int phstart = (int)floorf((float)(h - g.sh) / g.bin_h);
            int phend = (int)ceilf((float)(h - g.sh + 1) / g.bin_h);
            int pwstart = (int)floorf((float)(w - g.sw) / g.bin_w);
            int pwend = (int)ceilf((float)(w - g.sw + 1) / g.bin_w);
            phstart = std::min(std::max(phstart, 0), PH);
            phend = std::min(std::max(phend, 0), PH);
            pwstart = std::min(std::max(pwstart, 0), PW);
            pwend = std::min(std::max(pwend, 0), PW);
            size_t off = (size_t)r * PH * PW * Cout;
            for (int ph = phstart; ph < phend; ph++)
              for (int pw = pwstart; pw < pwend; pw++) {
                size_t t = off + ((size_t)ph * PW + pw) * Cout + (pool_channel ? 0 : c);
                if (argmax[t] == (h * W + w) * C + c) gradient += top_diff[t];
              }
          }
          bottom_diff[(((size_t)n * H + h) * W + w) * C + c] = gradient;
        }
  return 0;
}
