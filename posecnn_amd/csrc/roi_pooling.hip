// RoI max pooling for PoseCNN on MI355X (gfx950).
//
// Replaces ROIPoolForwardLaucher / ROIPoolBackwardLaucher
// (lib/roi_pooling_layer/roi_pooling_op_gpu.cu.cc:19-131 / :134-254).
//
// Forward: one workgroup per (RoI, output row ph); lanes run over channels, so
// every bin read is a coalesced sweep of the NHWC channel vector.  Bin bounds,
// rounding (roundf = half away from zero) and the strict-> first-max argmax
// follow cu.cc:45-97 exactly.
//
// Backward: the reference gives every bottom element one thread that loops
// over ALL RoIs (O(B*H*W*C*R), cu.cc:134-229).  Here one wave owns one bottom
// pixel and all its channels; the RoI loop is wave-uniform, restricted to the
// RoIs of that image (per-image [first, last] ranges from a prep kernel) and to
// the 1-4 bins whose range contains the pixel.  Contributions are added in the
// reference's order (RoI ascending, ph, pw), so the fp32 sums are bit-equal.
#include "pcnn_common.h"
#include <math.h>
#include <cfloat>

namespace {

struct RoiGeo {
  int b, cls, sw, sh, ew, eh;
  float bin_h, bin_w;
};

__device__ __forceinline__ RoiGeo roi_geo(const float* __restrict__ rois, int r, int stride, float scale, int PH,
                                          int PW) {
  const float* o = rois + (size_t)r * stride;
  RoiGeo g;
  g.b = (int)o[0];
  const int c0 = stride == 5 ? 1 : 2;
  g.cls = stride == 5 ? 0 : (int)o[1];
  g.sw = (int)roundf(o[c0 + 0] * scale);
  g.sh = (int)roundf(o[c0 + 1] * scale);
  g.ew = (int)roundf(o[c0 + 2] * scale);
  g.eh = (int)roundf(o[c0 + 3] * scale);
  const int roi_w = max(g.ew - g.sw + 1, 1);
  const int roi_h = max(g.eh - g.sh + 1, 1);
  g.bin_h = (float)roi_h / (float)PH;
  g.bin_w = (float)roi_w / (float)PW;
  return g;
}

__device__ __forceinline__ int rows_of(const int32_t* num_rois_dev, int R_cap) {
  if (!num_rois_dev) return R_cap;
  int r = *num_rois_dev;
  return r < R_cap ? r : R_cap;
}

// cu.cc:61-74
__device__ __forceinline__ void bin_bounds(const RoiGeo& g, int ph, int pw, int H, int W, int& hs, int& he, int& ws,
                                           int& we) {
  hs = (int)floorf((float)ph * g.bin_h);
  ws = (int)floorf((float)pw * g.bin_w);
  he = (int)ceilf((float)(ph + 1) * g.bin_h);
  we = (int)ceilf((float)(pw + 1) * g.bin_w);
  hs = min(max(hs + g.sh, 0), H);
  he = min(max(he + g.sh, 0), H);
  ws = min(max(ws + g.sw, 0), W);
  we = min(max(we + g.sw, 0), W);
}

// NHWC, all channels: block (roi, ph), threads over channels
__global__ void __launch_bounds__(256) k_roi_fwd_nhwc(const float* __restrict__ data, int B, int H, int W, int C,
                                                       const float* __restrict__ rois, int R_cap, int stride,
                                                       const int32_t* __restrict__ num_rois_dev, float scale, int PH,
                                                       int PW, float* __restrict__ top, int32_t* __restrict__ argmax) {
  const int r = blockIdx.x, ph = blockIdx.y;
  if (r >= rows_of(num_rois_dev, R_cap)) return;
  const RoiGeo g = roi_geo(rois, r, stride, scale, PH, PW);
  const bool bad = g.b < 0 || g.b >= B;
  const float* bd = data + (size_t)(bad ? 0 : g.b) * H * W * C;
  for (int pw = 0; pw < PW; pw++) {
    int hs, he, ws, we;
    bin_bounds(g, ph, pw, H, W, hs, he, ws, we);
    const bool empty = bad || (he <= hs) || (we <= ws);
    float* to = top + (((size_t)r * PH + ph) * PW + pw) * C;
    int32_t* ao = argmax + (((size_t)r * PH + ph) * PW + pw) * C;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float maxval = empty ? 0.f : -FLT_MAX;
      int maxidx = -1;
      if (!empty)
        for (int h = hs; h < he; h++)
          for (int w = ws; w < we; w++) {
            const int bi = (h * W + w) * C + c;
            const float v = bd[bi];
            if (v > maxval) { maxval = v; maxidx = bi; }
          }
      to[c] = maxval;
      ao[c] = maxidx;
    }
  }
}

// generic: one thread per output element (NCHW layout, or pool_channel)
__global__ void k_roi_fwd_generic(const float* __restrict__ data, int B, int H, int W, int C, int layout,
                                  const float* __restrict__ rois, int R_cap, int stride,
                                  const int32_t* __restrict__ num_rois_dev, float scale, int PH, int PW,
                                  int pool_channel, float* __restrict__ top, int32_t* __restrict__ argmax) {
  const int R = rows_of(num_rois_dev, R_cap);
  const int Co = pool_channel ? 1 : C;
  const long n_out = (long)R * PH * PW * Co;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n_out; idx += (long)gridDim.x * blockDim.x) {
    int r, ph, pw, c;
    if (layout == 0) {  // (R, PH, PW, Co)
      long t = idx;
      c = (int)(t % Co); t /= Co;
      pw = (int)(t % PW); t /= PW;
      ph = (int)(t % PH); r = (int)(t / PH);
    } else {  // (R, Co, PH, PW)
      long t = idx;
      pw = (int)(t % PW); t /= PW;
      ph = (int)(t % PH); t /= PH;
      c = (int)(t % Co); r = (int)(t / Co);
    }
    const RoiGeo g = roi_geo(rois, r, stride, scale, PH, PW);
    const bool bad = g.b < 0 || g.b >= B;
    const int ch = pool_channel ? g.cls : c;
    int hs, he, ws, we;
    bin_bounds(g, ph, pw, H, W, hs, he, ws, we);
    const bool empty = bad || (he <= hs) || (we <= ws) || ch < 0 || ch >= C;
    float maxval = empty ? 0.f : -FLT_MAX;
    int maxidx = -1;
    if (!empty) {
      const float* bd = data + (size_t)g.b * H * W * C;
      for (int h = hs; h < he; h++)
        for (int w = ws; w < we; w++) {
          const int bi = layout == 0 ? (h * W + w) * C + ch : (ch * H + h) * W + w;
          const float v = bd[bi];
          if (v > maxval) { maxval = v; maxidx = bi; }
        }
    }
    top[idx] = maxval;
    argmax[idx] = maxidx;
  }
}

// per-image RoI index ranges (rois may come in any order; ranges bound the scan)
__global__ void k_roi_ranges(const float* __restrict__ rois, int R_cap, int stride,
                             const int32_t* __restrict__ num_rois_dev, int B, int32_t* __restrict__ lo,
                             int32_t* __restrict__ hi) {
  const int R = rows_of(num_rois_dev, R_cap);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    lo[b] = 0x7fffffff;
    hi[b] = -1;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const int b = (int)rois[(size_t)r * stride];
    if (b >= 0 && b < B) {
      atomicMin(&lo[b], r);
      atomicMax(&hi[b], r);
    }
  }
}

// NHWC all-channel backward: one wave per bottom pixel (b, h, w)
__global__ void __launch_bounds__(256) k_roi_bwd_nhwc(const float* __restrict__ top_diff,
                                                       const int32_t* __restrict__ argmax, int B, int H, int W, int C,
                                                       const float* __restrict__ rois, int stride, float scale,
                                                       int PH, int PW, const int32_t* __restrict__ lo,
                                                       const int32_t* __restrict__ hi, float* __restrict__ bottom) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = pcnn::lane_id();
  if (wave >= B * H * W) return;
  const int w = wave % W, h = (wave / W) % H, b = wave / (W * H);
  float* bo = bottom + (size_t)wave * C;
  const int pix = (h * W + w) * C;
  const int r0 = lo[b], r1 = hi[b];
  for (int c0 = 0; c0 < C; c0 += 64 * 4) {
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = r0; r <= r1; r++) {
      const RoiGeo gg = roi_geo(rois, r, stride, scale, PH, PW);
      if (gg.b != b) continue;
      if (!(w >= gg.sw && w <= gg.ew && h >= gg.sh && h <= gg.eh)) continue;  // cu.cc:172-177
      int phs = (int)floorf((float)(h - gg.sh) / gg.bin_h);
      int phe = (int)ceilf((float)(h - gg.sh + 1) / gg.bin_h);
      int pws = (int)floorf((float)(w - gg.sw) / gg.bin_w);
      int pwe = (int)ceilf((float)(w - gg.sw + 1) / gg.bin_w);
      phs = min(max(phs, 0), PH);
      phe = min(max(phe, 0), PH);
      pws = min(max(pws, 0), PW);
      pwe = min(max(pwe, 0), PW);
      for (int ph = phs; ph < phe; ph++)
        for (int pw = pws; pw < pwe; pw++) {
          const size_t t = (((size_t)r * PH + ph) * PW + pw) * C;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int c = c0 + k * 64 + lane;
            if (c < C && argmax[t + c] == pix + c) g[k] += top_diff[t + c];
          }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int c = c0 + k * 64 + lane;
      if (c < C) bo[c] = g[k];
    }
  }
}

// generic backward (NCHW layout or pool_channel): one thread per bottom pixel
// owns every channel of it; RoIs ascending keeps the per-channel order.
__global__ void k_roi_bwd_generic(const float* __restrict__ top_diff, const int32_t* __restrict__ argmax, int B,
                                  int H, int W, int C, int layout, const float* __restrict__ rois, int stride,
                                  float scale, int PH, int PW, int pool_channel, const int32_t* __restrict__ lo,
                                  const int32_t* __restrict__ hi, float* __restrict__ bottom) {
  const long npix = (long)B * H * W;
  const int Co = pool_channel ? 1 : C;
  for (long pi = (long)blockIdx.x * blockDim.x + threadIdx.x; pi < npix; pi += (long)gridDim.x * blockDim.x) {
    const int w = (int)(pi % W), h = (int)((pi / W) % H), b = (int)(pi / ((long)W * H));
    const int r0 = lo[b], r1 = hi[b];
    for (int r = r0; r <= r1; r++) {
      const RoiGeo gg = roi_geo(rois, r, stride, scale, PH, PW);
      if (gg.b != b) continue;
      if (!(w >= gg.sw && w <= gg.ew && h >= gg.sh && h <= gg.eh)) continue;
      int phs = (int)floorf((float)(h - gg.sh) / gg.bin_h);
      int phe = (int)ceilf((float)(h - gg.sh + 1) / gg.bin_h);
      int pws = (int)floorf((float)(w - gg.sw) / gg.bin_w);
      int pwe = (int)ceilf((float)(w - gg.sw + 1) / gg.bin_w);
      phs = min(max(phs, 0), PH);
      phe = min(max(phe, 0), PH);
      pws = min(max(pws, 0), PW);
      pwe = min(max(pwe, 0), PW);
      const int cb = pool_channel ? gg.cls : 0, ce = pool_channel ? gg.cls + 1 : C;
      if (cb < 0 || ce > C) continue;
      for (int c = cb; c < ce; c++) {
        const int bidx = layout == 0 ? (h * W + w) * C + c : (c * H + h) * W + w;
        float* dst = bottom + (size_t)b * H * W * C + bidx;
        float acc = *dst;
        for (int ph = phs; ph < phe; ph++)
          for (int pw = pws; pw < pwe; pw++) {
            const int oc = pool_channel ? 0 : c;
            const size_t t = layout == 0 ? (((size_t)r * PH + ph) * PW + pw) * Co + oc
                                         : (((size_t)r * Co + oc) * PH + ph) * PW + pw;
            if (argmax[t] == bidx) acc += top_diff[t];
          }
        *dst = acc;
      }
    }
  }
}

}  // namespace

extern "C" int pcnn_roi_pool_fwd(const float* data, int B, int H, int W, int C, int layout, const float* rois,
                                 int R_cap, int roi_stride, const int32_t* num_rois_dev, float spatial_scale,
                                 int pooled_h, int pooled_w, int pool_channel, float* top, int32_t* argmax,
                                 void* stream) {
  PCNN_REQUIRE(data && rois && top && argmax && B > 0 && H > 0 && W > 0 && C > 0 && R_cap >= 0);
  PCNN_REQUIRE(pooled_h > 0 && pooled_w > 0 && (layout == 0 || layout == 1));
  PCNN_REQUIRE(roi_stride >= 6 || (roi_stride == 5 && !pool_channel));
  PCNN_REQUIRE((long)H * W * C < (1l << 31));
  if (R_cap == 0) return PCNN_OK;
  hipStream_t st = (hipStream_t)stream;
  if (layout == 0 && !pool_channel) {
    hipLaunchKernelGGL(k_roi_fwd_nhwc, dim3(R_cap, pooled_h), dim3(C >= 256 ? 256 : (C + 63) / 64 * 64), 0, st, data,
                       B, H, W, C, rois, R_cap, roi_stride, num_rois_dev, spatial_scale, pooled_h, pooled_w, top,
                       argmax);
  } else {
    const long n = (long)R_cap * pooled_h * pooled_w * (pool_channel ? 1 : C);
    const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_fwd_generic, dim3(blocks), dim3(256), 0, st, data, B, H, W, C, layout, rois, R_cap,
                       roi_stride, num_rois_dev, spatial_scale, pooled_h, pooled_w, pool_channel, top, argmax);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" size_t pcnn_roi_pool_bwd_workspace_size(int B, int R_cap) {
  (void)R_cap;
  return pcnn::align_up((size_t)2 * (B > 0 ? B : 1) * sizeof(int32_t), 256) + 256;
}

extern "C" int pcnn_roi_pool_bwd(const float* top_diff, const int32_t* argmax, int B, int H, int W, int C, int layout,
                                 const float* rois, int R_cap, int roi_stride, const int32_t* num_rois_dev,
                                 float spatial_scale, int pooled_h, int pooled_w, int pool_channel,
                                 float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(top_diff && argmax && rois && bottom_diff && workspace && B > 0 && H > 0 && W > 0 && C > 0);
  PCNN_REQUIRE(pooled_h > 0 && pooled_w > 0 && (layout == 0 || layout == 1));
  PCNN_REQUIRE(roi_stride >= 6 || (roi_stride == 5 && !pool_channel));
  PCNN_REQUIRE((long)H * W * C < (1l << 31));
  if (workspace_bytes < pcnn_roi_pool_bwd_workspace_size(B, R_cap)) return PCNN_ECAPACITY;
  hipStream_t st = (hipStream_t)stream;
  int32_t* lo = (int32_t*)workspace;
  int32_t* hi = lo + B;
  hipLaunchKernelGGL(k_roi_ranges, dim3(1), dim3(1024), 0, st, rois, R_cap, roi_stride, num_rois_dev, B, lo, hi);
  if (layout == 0 && !pool_channel) {
    const long waves = (long)B * H * W;
    hipLaunchKernelGGL(k_roi_bwd_nhwc, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, top_diff, argmax, B, H, W,
                       C, rois, roi_stride, spatial_scale, pooled_h, pooled_w, lo, hi, bottom_diff);
  } else {
    if (hipMemsetAsync(bottom_diff, 0, (size_t)B * H * W * C * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
    const long npix = (long)B * H * W;
    const int blocks = (int)((npix + 255) / 256 < 8192 ? (npix + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_bwd_generic, dim3(blocks), dim3(256), 0, st, top_diff, argmax, B, H, W, C, layout, rois,
                       roi_stride, spatial_scale, pooled_h, pooled_w, pool_channel, lo, hi, bottom_diff);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
