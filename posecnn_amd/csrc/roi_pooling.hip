// RoI max pooling for PoseCNN on MI355X (gfx950).
//
// Replaces ROIPoolForwardLaucher / ROIPoolBackwardLaucher
// (lib/roi_pooling_layer/roi_pooling_op_gpu.cu.cc:19-131 / :134-254).
//
// Forward (NHWC, all channels): one workgroup per (RoI, bin); each lane owns a
// float4 of channels, so every bin pixel is one coalesced 16 B-per-lane sweep
// of the channel vector and a bin's pixel loads are independent (issued back
// to back).  Bin bounds, rounding (roundf = half away from zero) and the
// strict-> first-max argmax follow cu.cc:45-97 exactly.
//
// Backward: the reference gives every bottom element one thread that loops
// over ALL RoIs (O(B*H*W*C*R), cu.cc:134-229).  Here the RoI geometry is
// computed once (k_roi_prep); each workgroup owns a 2x4 pixel tile of one
// image and a 128-channel chunk, lists the (RoI, ph, pw) entries whose bins
// can feed the tile in the reference's order (RoI ascending, ph, pw), reads
// each entry once and accumulates the argmax-matching top gradients per tile
// pixel in registers — the fp32 sums are bit-equal to the reference kernel's.
#include "pcnn_common.h"
#include <math.h>
#include <cfloat>

namespace {


struct RoiGeo {
  int b, cls, sw, sh, ew, eh;
  float bin_h, bin_w;
};

// batch_base: the rows' batch column holds the global image index in an
// image-sharded run (hough emit adds it, hough_common.h); the feature maps
// hold only this rank's images, so the map index is column - batch_base.
__device__ __forceinline__ RoiGeo roi_geo(const float* __restrict__ rois, int r, int stride, int batch_base,
                                          float scale, int PH, int PW) {
  const float* o = rois + (size_t)r * stride;
  RoiGeo g;
  g.b = (int)o[0] - batch_base;
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

// cu.cc:196-204: bins of one RoI whose range can contain (h, w)
__device__ __forceinline__ void bins_of_pixel(const RoiGeo& g, int h, int w, int PH, int PW, int& phs, int& phe,
                                              int& pws, int& pwe) {
  phs = (int)floorf((float)(h - g.sh) / g.bin_h);
  phe = (int)ceilf((float)(h - g.sh + 1) / g.bin_h);
  pws = (int)floorf((float)(w - g.sw) / g.bin_w);
  pwe = (int)ceilf((float)(w - g.sw + 1) / g.bin_w);
  phs = min(max(phs, 0), PH);
  phe = min(max(phe, 0), PH);
  pws = min(max(pws, 0), PW);
  pwe = min(max(pwe, 0), PW);
}

__device__ __forceinline__ void upd(float v, int idx, float& m, int& a) {
  if (v > m) { m = v; a = idx; }
}

// XCD-aware (row, bin) of a forward workgroup.  Workgroups are dealt
// round-robin to the 8 XCDs, each with its own L2.  Rows go to the XCDs in
// runs of kRun = 9 (one object's box and its 8 jitters in train mode,
// cu.cc:469-554), with a run's bins consecutive, so a RoI's feature window is
// fetched into one L2 and re-read there by its jittered neighbours instead of
// by all eight XCDs.  Same box, B = 8 bench RoIs: the pool pair 94.6 -> 60 us
// (PCNN_ROI_XCD=0 is the plain row-fastest order, kept for A/B).
#ifndef PCNN_ROI_XCD
#define PCNN_ROI_XCD 1
#endif
constexpr int kXcds = 8;
constexpr int kRun = 9;
__device__ __forceinline__ bool fwd_item(int R, int nbins, int& r, int& bin) {
  const int id = blockIdx.x;
#if PCNN_ROI_XCD
  const int x = id % kXcds, local = id / kXcds;
  const int lr = local / nbins;
  bin = local % nbins;
  r = ((lr / kRun) * kXcds + x) * kRun + lr % kRun;
#else
  const int rows = gridDim.x / nbins;
  r = id % rows;
  bin = id / rows;
#endif
  return r < R;
}
// 1-D grid: whole runs on every XCD
static inline unsigned fwd_grid(int R_cap, int nbins) {
  return (unsigned)(kXcds * ((R_cap + kXcds * kRun - 1) / (kXcds * kRun)) * kRun * nbins);
}

// Max / argmax of one bin over lane channels c..c+3 (cu.cc:45-97): bin
// bounds as bin_bounds, strict > first max in raster order, empty bin (or a
// RoI batch index outside [0, B)) -> 0 / -1.
// PX: the argmax is the pixel index h * W + w within the image (the channel is
// the output's own), the compact form of the fused pose step.
template <bool PX = false>
__device__ __forceinline__ void bin_max4(const float* __restrict__ data, int B, int H, int W, int C,
                                         const RoiGeo& g, int ph, int pw, int c, float4& m, int4& a) {
  const bool bad = g.b < 0 || g.b >= B;
  int hs, he, ws, we;
  bin_bounds(g, ph, pw, H, W, hs, he, ws, we);
  const bool empty = bad || (he <= hs) || (we <= ws);
  const float* bd = data + (size_t)(bad ? 0 : g.b) * H * W * C;
  float m0, m1, m2, m3;
  m0 = m1 = m2 = m3 = empty ? 0.f : -FLT_MAX;
  int a0 = -1, a1 = -1, a2 = -1, a3 = -1;
  if (!empty) {
    for (int h = hs; h < he; h++) {
      int w = ws;
      for (; w + 1 < we; w += 2) {  // two independent 16 B loads in flight
        const int i0 = (h * W + w) * C + c, i1 = i0 + C;
        const float4 v0 = *(const float4*)(bd + i0);
        const float4 v1 = *(const float4*)(bd + i1);
        if (PX) {
          const int p0 = h * W + w, p1 = p0 + 1;
          upd(v0.x, p0, m0, a0); upd(v0.y, p0, m1, a1); upd(v0.z, p0, m2, a2); upd(v0.w, p0, m3, a3);
          upd(v1.x, p1, m0, a0); upd(v1.y, p1, m1, a1); upd(v1.z, p1, m2, a2); upd(v1.w, p1, m3, a3);
        } else {
          upd(v0.x, i0 + 0, m0, a0); upd(v0.y, i0 + 1, m1, a1); upd(v0.z, i0 + 2, m2, a2); upd(v0.w, i0 + 3, m3, a3);
          upd(v1.x, i1 + 0, m0, a0); upd(v1.y, i1 + 1, m1, a1); upd(v1.z, i1 + 2, m2, a2); upd(v1.w, i1 + 3, m3, a3);
        }
      }
      if (w < we) {
        const int i0 = (h * W + w) * C + c;
        const float4 v0 = *(const float4*)(bd + i0);
        if (PX) {
          const int p0 = h * W + w;
          upd(v0.x, p0, m0, a0); upd(v0.y, p0, m1, a1); upd(v0.z, p0, m2, a2); upd(v0.w, p0, m3, a3);
        } else {
          upd(v0.x, i0 + 0, m0, a0); upd(v0.y, i0 + 1, m1, a1); upd(v0.z, i0 + 2, m2, a2); upd(v0.w, i0 + 3, m3, a3);
        }
      }
    }
  }
  m = make_float4(m0, m1, m2, m3);
  a = make_int4(a0, a1, a2, a3);
}

// NHWC, all channels, C % 4 == 0: block (roi, bin), lane -> 4 channels.
// ACC: top += pooled (the pool5 + pool4 sum of vgg16_convs.py:184 produced in
// place by the second pool; the argmax of each map is still written).
template <bool ACC>
__global__ void __launch_bounds__(128) k_roi_fwd_nhwc4(const float* __restrict__ data, int B, int H, int W, int C,
                                                        const float* __restrict__ rois, int R_cap, int stride,
                                                        int batch_base, const int32_t* __restrict__ num_rois_dev,
                                                        float scale, int PH, int PW, float* __restrict__ top,
                                                        int32_t* __restrict__ argmax) {
  int r, bin;
  if (!fwd_item(rows_of(num_rois_dev, R_cap), PH * PW, r, bin)) return;
  const int ph = bin / PW, pw = bin % PW;
  const RoiGeo g = roi_geo(rois, r, stride, batch_base, scale, PH, PW);
  float* to = top + (((size_t)r * PH + ph) * PW + pw) * C;
  int32_t* ao = argmax + (((size_t)r * PH + ph) * PW + pw) * C;
  for (int c = threadIdx.x * 4; c < C; c += blockDim.x * 4) {
    float4 m;
    int4 a;
    bin_max4(data, B, H, W, C, g, ph, pw, c, m, a);
    if (ACC) {
      const float4 p = *(const float4*)(to + c);
      *(float4*)(to + c) = make_float4(p.x + m.x, p.y + m.y, p.z + m.z, p.w + m.w);
    } else {
      *(float4*)(to + c) = m;
    }
    *(int4*)(ao + c) = a;
  }
}

// Both RoI pools of the pose head in one pass (vgg16_convs.py:177-184:
// pool5 on conv5_3 at 1/16, pool4 on conv4_3 at 1/8, then their sum): block
// (roi, bin) takes the bin on both maps, so the two maps' loads are in flight
// together, and writes pool5 + pool4 (the same single fp32 add as the
// accumulate pass) and both argmax tensors — no pool5 round trip through HBM.
// PX: argmax as uint16 pixel indices (h * W + w; 0xFFFF = empty bin), half the
// argmax bytes written here and read back by k_roi_bwd_ent<.., true>.
template <bool PX>
__global__ void __launch_bounds__(128) k_roi_fwd_pair_nhwc4(const float* __restrict__ data_a, int Ha, int Wa,
                                                             float scale_a, const float* __restrict__ data_b, int Hb,
                                                             int Wb, float scale_b, int B, int C,
                                                             const float* __restrict__ rois, int R_cap, int stride,
                                                             int batch_base, const int32_t* __restrict__ num_rois_dev,
                                                             int PH, int PW, float* __restrict__ top,
                                                             void* __restrict__ arg_a, void* __restrict__ arg_b) {
  int r, bin;
  if (!fwd_item(rows_of(num_rois_dev, R_cap), PH * PW, r, bin)) return;
  const int ph = bin / PW, pw = bin % PW;
  const RoiGeo ga = roi_geo(rois, r, stride, batch_base, scale_a, PH, PW);
  const RoiGeo gb = roi_geo(rois, r, stride, batch_base, scale_b, PH, PW);
  const size_t o = (((size_t)r * PH + ph) * PW + pw) * C;
  for (int c = threadIdx.x * 4; c < C; c += blockDim.x * 4) {
    float4 ma, mb;
    int4 aa, ab;
    bin_max4<PX>(data_a, B, Ha, Wa, C, ga, ph, pw, c, ma, aa);
    bin_max4<PX>(data_b, B, Hb, Wb, C, gb, ph, pw, c, mb, ab);
    *(float4*)(top + o + c) = make_float4(ma.x + mb.x, ma.y + mb.y, ma.z + mb.z, ma.w + mb.w);
    if (PX) {
      auto pk = [](int4 a) {  // -1 -> 0xFFFF
        return make_uint2(((unsigned)a.x & 0xFFFFu) | ((unsigned)a.y << 16),
                          ((unsigned)a.z & 0xFFFFu) | ((unsigned)a.w << 16));
      };
      *(uint2*)((uint16_t*)arg_a + o + c) = pk(aa);
      *(uint2*)((uint16_t*)arg_b + o + c) = pk(ab);
    } else {
      *(int4*)((int32_t*)arg_a + o + c) = aa;
      *(int4*)((int32_t*)arg_b + o + c) = ab;
    }
  }
}

// generic: one thread per output element (NCHW layout, pool_channel, C % 4 != 0)
__global__ void k_roi_fwd_generic(const float* __restrict__ data, int B, int H, int W, int C, int layout,
                                  const float* __restrict__ rois, int R_cap, int stride, int batch_base,
                                  const int32_t* __restrict__ num_rois_dev, float scale, int PH, int PW,
                                  int pool_channel, int acc, float* __restrict__ top, int32_t* __restrict__ argmax) {
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
    const RoiGeo g = roi_geo(rois, r, stride, batch_base, scale, PH, PW);
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
    top[idx] = acc ? top[idx] + maxval : maxval;
    argmax[idx] = maxidx;
  }
}

// RoI geometry once per row + per-image RoI index ranges.
// geo[r] = {b, cls, sw, sh, ew, eh, bits(bin_h), bits(bin_w)}
__global__ void __launch_bounds__(1024) k_roi_prep(const float* __restrict__ rois, int R_cap, int stride,
                                                    int batch_base, const int32_t* __restrict__ num_rois_dev, int B,
                                                    float scale, int PH, int PW, int32_t* __restrict__ geo,
                                                    int32_t* __restrict__ lo, int32_t* __restrict__ hi) {
  __shared__ int slo[1024], shi[1024];
  const int R = rows_of(num_rois_dev, R_cap);
  const int nb = B < 1024 ? B : 1024;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    slo[b] = 0x7fffffff;
    shi[b] = -1;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const RoiGeo g = roi_geo(rois, r, stride, batch_base, scale, PH, PW);
    int32_t* o = geo + (size_t)r * 8;
    o[0] = g.b; o[1] = g.cls; o[2] = g.sw; o[3] = g.sh; o[4] = g.ew; o[5] = g.eh;
    o[6] = __float_as_int(g.bin_h);
    o[7] = __float_as_int(g.bin_w);
    if (g.b >= 0 && g.b < nb) {
      atomicMin(&slo[g.b], r);
      atomicMax(&shi[g.b], r);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    lo[b] = b < nb ? slo[b] : 0;
    hi[b] = b < nb ? shi[b] : -1;
  }
}

// NHWC all-channel backward, C % 2 == 0: one wave per (image, 2 x 4 pixel
// tile, 128-channel chunk), two channels per lane.  The
// reference gathers, per bottom element, over every RoI and every bin that can
// hold it (cu.cc:134-229); here the work is turned around.  Wave 0 lists the
// (RoI, ph, pw) entries whose bins can feed the tile — RoIs ascending, then
// ph, then pw: the reference's summation order — each with the 8-bit mask of
// tile pixels that pass the reference's own membership tests for it (inside
// the RoI box, ph in [phstart, phend), pw in [pwstart, pwend),
// cu.cc:172-204).  It then reads each listed entry's argmax / top
// gradient once (8 B per lane per operand, two batches of kBBatch entries in
// flight: the next batch loads while the current one accumulates) and,
// for every masked tile pixel, add the top gradient of each channel whose
// argmax names that pixel to a register accumulator (cu.cc:219-224) — in
// list order, so the fp32 sums are bit-equal to the reference's.
#ifndef PCNN_RBW_XCD
#define PCNN_RBW_XCD 1
#endif
#ifndef PCNN_RBW_NARROW
#define PCNN_RBW_NARROW 8192
#endif
constexpr int kBWaves = 1;  // one wave per workgroup: a tile's channel chunks land on different CUs
constexpr int kBChunk = 128 * kBWaves;  // channels per workgroup
constexpr int kBGroup = 16;             // RoIs expanded per list round (<= 16 * 49 entries)
constexpr int kBCap = kBGroup * 49;
constexpr int kBBatch = 8;              // entries per fetch (two fetches in flight per wave)

template <int kBTH, int kBTW, bool PX>
__global__ void __launch_bounds__(64 * kBWaves) k_roi_bwd_ent(const float* __restrict__ top_diff,
                                                               const void* __restrict__ argmax, int B, int H, int W,
                                                               int C, const int32_t* __restrict__ geo,
                                                               const int32_t* __restrict__ lo,
                                                               const int32_t* __restrict__ hi, int PH, int PW,
                                                               float* __restrict__ bottom) {
  constexpr int kBPix = kBTH * kBTW;
  __shared__ int2 ent[kBCap];  // element offset ((r*PH+ph)*PW+pw)*C, pixel mask
  __shared__ int sh_total;
  const int tiles_w = (W + kBTW - 1) / kBTW, tiles_h = (H + kBTH - 1) / kBTH;
  const int nchunk = (C + kBChunk - 1) / kBChunk;
#if PCNN_RBW_XCD
  // XCD-aware: XCD x takes the contiguous item range [x*ipx, (x+1)*ipx), so
  // neighbouring tiles, which list the same RoI bins, read them through one L2
  const int ipx = (int)((gridDim.x + 7) / 8);
  int id = (int)(blockIdx.x % 8) * ipx + (int)(blockIdx.x / 8);
#else
  int id = blockIdx.x;
#endif
  if (id >= B * tiles_w * tiles_h * nchunk) return;  // grid padded to a multiple of 8
  const int chunk = id % nchunk;
  id /= nchunk;
  const int t = id % (tiles_w * tiles_h), b = id / (tiles_w * tiles_h);
  const int h0 = (t / tiles_w) * kBTH, w0 = (t % tiles_w) * kBTW;
  const int th = min(kBTH, H - h0), tw = min(kBTW, W - w0);
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  const int c = chunk * kBChunk + 2 * threadIdx.x;  // this lane's channels c, c + 1
  const bool cok = c < C;
  float2 acc[kBPix];  // this lane's channels at the tile pixels
  int expv[kBPix];    // the argmax value that names each tile pixel for channel c (cu.cc:219-224)
#pragma unroll
  for (int p = 0; p < kBPix; p++) {
    acc[p] = make_float2(0.f, 0.f);
    const int pix = (h0 + p / kBTW) * W + w0 + p % kBTW;
    expv[p] = PX ? pix : pix * C + c;  // PX: pixel index, the same for both channels
  }
  constexpr int kNext = PX ? 0 : 1;  // argmax of channel c + 1 is expv + kNext
  const int r0 = lo[b], r1 = hi[b];
  // buffer views: per-lane channel offset in a VGPR, the entry offset as the
  // scalar soffset; lanes past C read out of range (-> 0 / never a match)
  const __amdgpu_buffer_rsrc_t rs_t = __builtin_amdgcn_make_buffer_rsrc((void*)top_diff, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_a = __builtin_amdgcn_make_buffer_rsrc((void*)argmax, (short)0, 0x7fffffff, 0x00020000);
  const unsigned voff = cok ? (unsigned)c * 4u : 0x80000000u;
  const unsigned voff_a = cok ? (unsigned)c * (PX ? 2u : 4u) : 0x80000000u;
  for (int rb = r0; rb <= r1; rb += 64) {
    // wave 0: RoIs of image b whose box meets the tile, in order (cu.cc:154-177),
    // with per-bin row / column acceptance bits for the tile pixels (cu.cc:196-204)
    uint32_t rbits = 0;  // bit (ph * kBTH + i): tile row i accepts bin row ph
    uint32_t cbits = 0;  // bit (pw * kBTW + j): tile col j accepts bin col pw
    const int r = rb + lane;
    if (wave == 0 && r <= r1) {
      const int32_t* gg = geo + (size_t)r * 8;
      RoiGeo g;
      g.b = gg[0]; g.sw = gg[2]; g.sh = gg[3]; g.ew = gg[4]; g.eh = gg[5];
      g.bin_h = __int_as_float(gg[6]);
      g.bin_w = __int_as_float(gg[7]);
      if (g.b == b && g.sh <= h0 + th - 1 && g.eh >= h0 && g.sw <= w0 + tw - 1 && g.ew >= w0) {
        for (int i = 0; i < th; i++) {
          const int h = h0 + i;
          if (h < g.sh || h > g.eh) continue;
          int s0 = (int)floorf((float)(h - g.sh) / g.bin_h), e0 = (int)ceilf((float)(h - g.sh + 1) / g.bin_h);
          s0 = min(max(s0, 0), PH);
          e0 = min(max(e0, 0), PH);
          for (int ph = s0; ph < e0; ph++) rbits |= 1u << (ph * kBTH + i);
        }
        for (int j = 0; j < tw; j++) {
          const int w = w0 + j;
          if (w < g.sw || w > g.ew) continue;
          int s0 = (int)floorf((float)(w - g.sw) / g.bin_w), e0 = (int)ceilf((float)(w - g.sw + 1) / g.bin_w);
          s0 = min(max(s0, 0), PW);
          e0 = min(max(e0, 0), PW);
          for (int pw = s0; pw < e0; pw++) cbits |= 1u << (pw * kBTW + j);
        }
      }
    }
    const uint64_t hits = __ballot(rbits && cbits);  // wave 0's view; 0 in the other wave
    for (int g0 = 0; g0 < 64; g0 += kBGroup) {
      if (wave == 0) {
        const uint64_t gm = hits & (((1ull << kBGroup) - 1) << g0);
        const bool mine = (gm >> lane) & 1;
        int cnt = 0;
        if (mine) {
          int nph = 0, npw = 0;
          for (int ph = 0; ph < PH; ph++) nph += ((rbits >> (ph * kBTH)) & ((1u << kBTH) - 1)) != 0;
          for (int pw = 0; pw < PW; pw++) npw += ((cbits >> (pw * kBTW)) & ((1u << kBTW) - 1)) != 0;
          cnt = nph * npw;
        }
        int off = cnt;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int v = __shfl_up(off, d, 64);
          if (lane >= d) off += v;
        }
        if (lane == 63) sh_total = off;
        off -= cnt;
        if (mine) {
          const int rbase = r * PH;
          for (int ph = 0; ph < PH; ph++) {
            const uint32_t rm = (rbits >> (ph * kBTH)) & ((1u << kBTH) - 1);
            if (!rm) continue;
            for (int pw = 0; pw < PW; pw++) {
              const uint32_t cm = (cbits >> (pw * kBTW)) & ((1u << kBTW) - 1);
              if (!cm) continue;
              uint32_t m = 0;
#pragma unroll
              for (int i = 0; i < kBTH; i++)
                if ((rm >> i) & 1) m |= cm << (i * kBTW);
              ent[off++] = make_int2(((rbase + ph) * PW + pw) * C, (int)m);
            }
          }
        }
      }
      __syncthreads();
      const int total = sh_total;
      // lane k reads entry e0 + k and hands its offset / mask to the wave
      auto fetch = [&](int e0, int2& my, int2 (&av)[kBBatch], float2 (&dv)[kBBatch]) {
        my = ent[min(e0 + (lane & (kBBatch - 1)), total - 1)];
#pragma unroll
        for (int k = 0; k < kBBatch; k++) {
          const int so = __builtin_amdgcn_readlane(my.x, k) * 4;
          if (PX) {  // two uint16 pixel indices (lanes past C read 0: they never store)
            const unsigned a2 = __builtin_amdgcn_raw_buffer_load_b32(rs_a, voff_a, so >> 1, 0);
            av[k] = make_int2((int)(a2 & 0xFFFFu), (int)(a2 >> 16));
          } else {
            av[k] = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(rs_a, voff_a, so, 0));
          }
          dv[k] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs_t, voff, so, 0));
        }
      };
      auto accumulate = [&](int e0, const int2& my, const int2 (&av)[kBBatch], const float2 (&dv)[kBBatch]) {
#pragma unroll
        for (int k = 0; k < kBBatch; k++) {
          if (e0 + k >= total) break;
          const uint32_t m = (uint32_t)__builtin_amdgcn_readlane(my.y, k);  // wave-uniform pixel mask
#pragma unroll
          for (int q = 0; q < kBPix; q++) {
            if (!((m >> q) & 1)) continue;
            // adding +0.0f leaves every partial sum bit-identical (none is ever -0)
            acc[q].x += av[k].x == expv[q] ? dv[k].x : 0.f;
            acc[q].y += av[k].y == expv[q] + kNext ? dv[k].y : 0.f;
          }
        }
      };
      if (total > 0) {
        int2 myA, myB, avA[kBBatch], avB[kBBatch];
        float2 dvA[kBBatch], dvB[kBBatch];
        fetch(0, myA, avA, dvA);
        for (int e0 = 0; e0 < total; e0 += 2 * kBBatch) {
          if (e0 + kBBatch < total) fetch(e0 + kBBatch, myB, avB, dvB);
          accumulate(e0, myA, avA, dvA);
          if (e0 + 2 * kBBatch < total) fetch(e0 + 2 * kBBatch, myA, avA, dvA);
          if (e0 + kBBatch < total) accumulate(e0 + kBBatch, myB, avB, dvB);
        }
      }
      __syncthreads();
    }
  }
  if (cok) {
#pragma unroll
    for (int i = 0; i < kBTH; i++)
#pragma unroll
      for (int j = 0; j < kBTW; j++)
        if (i < th && j < tw) *(float2*)(bottom + (((size_t)b * H + h0 + i) * W + w0 + j) * C + c) = acc[i * kBTW + j];
  }
}

// generic backward (NCHW layout, pool_channel, or C % 4 != 0): one thread per
// bottom pixel owns every channel of it; RoIs ascending keeps per-channel order.
__global__ void k_roi_bwd_generic(const float* __restrict__ top_diff, const int32_t* __restrict__ argmax, int B,
                                  int H, int W, int C, int layout, const int32_t* __restrict__ geo, int PH, int PW,
                                  int pool_channel, const int32_t* __restrict__ lo, const int32_t* __restrict__ hi,
                                  float* __restrict__ bottom) {
  const long npix = (long)B * H * W;
  const int Co = pool_channel ? 1 : C;
  for (long pi = (long)blockIdx.x * blockDim.x + threadIdx.x; pi < npix; pi += (long)gridDim.x * blockDim.x) {
    const int w = (int)(pi % W), h = (int)((pi / W) % H), b = (int)(pi / ((long)W * H));
    const int r0 = lo[b], r1 = hi[b];
    for (int r = r0; r <= r1; r++) {
      const int32_t* gg = geo + (size_t)r * 8;
      RoiGeo g;
      g.b = gg[0]; g.cls = gg[1]; g.sw = gg[2]; g.sh = gg[3]; g.ew = gg[4]; g.eh = gg[5];
      g.bin_h = __int_as_float(gg[6]);
      g.bin_w = __int_as_float(gg[7]);
      if (g.b != b) continue;
      if (!(w >= g.sw && w <= g.ew && h >= g.sh && h <= g.eh)) continue;
      int phs, phe, pws, pwe;
      bins_of_pixel(g, h, w, PH, PW, phs, phe, pws, pwe);
      const int cb = pool_channel ? g.cls : 0, ce = pool_channel ? g.cls + 1 : C;
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

static int roi_pool_fwd(const float* data, int B, int H, int W, int C, int layout, const float* rois, int R_cap,
                        int roi_stride, int batch_base, const int32_t* num_rois_dev, float spatial_scale,
                        int pooled_h, int pooled_w, int pool_channel, int acc, float* top, int32_t* argmax,
                        void* stream) {
  PCNN_REQUIRE(data && rois && top && argmax && B > 0 && H > 0 && W > 0 && C > 0 && R_cap >= 0);
  PCNN_REQUIRE(pooled_h > 0 && pooled_w > 0 && (layout == 0 || layout == 1));
  PCNN_REQUIRE(roi_stride >= 6 || (roi_stride == 5 && !pool_channel));
  PCNN_REQUIRE((long)H * W * C < (1l << 31));
  if (R_cap == 0) return PCNN_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = layout == 0 && !pool_channel && C % 4 == 0 && (((uintptr_t)data | (uintptr_t)top |
                                                                    (uintptr_t)argmax) & 15) == 0;
  if (vec) {
    const int threads = C / 4 >= 128 ? 128 : ((C / 4 + 63) / 64) * 64;
    if (acc)
      hipLaunchKernelGGL(k_roi_fwd_nhwc4<true>, dim3(fwd_grid(R_cap, pooled_h * pooled_w)), dim3(threads), 0, st, data, B, H,
                         W, C, rois, R_cap, roi_stride, batch_base, num_rois_dev, spatial_scale, pooled_h, pooled_w, top,
                         argmax);
    else
      hipLaunchKernelGGL(k_roi_fwd_nhwc4<false>, dim3(fwd_grid(R_cap, pooled_h * pooled_w)), dim3(threads), 0, st, data, B, H,
                         W, C, rois, R_cap, roi_stride, batch_base, num_rois_dev, spatial_scale, pooled_h, pooled_w, top,
                         argmax);
  } else {
    const long n = (long)R_cap * pooled_h * pooled_w * (pool_channel ? 1 : C);
    const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_fwd_generic, dim3(blocks), dim3(256), 0, st, data, B, H, W, C, layout, rois, R_cap,
                       roi_stride, batch_base, num_rois_dev, spatial_scale, pooled_h, pooled_w, pool_channel, acc, top,
                       argmax);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_roi_pool_fwd(const float* data, int B, int H, int W, int C, int layout, const float* rois,
                                 int R_cap, int roi_stride, int batch_base, const int32_t* num_rois_dev,
                                 float spatial_scale, int pooled_h, int pooled_w, int pool_channel, float* top,
                                 int32_t* argmax, void* stream) {
  return roi_pool_fwd(data, B, H, W, C, layout, rois, R_cap, roi_stride, batch_base, num_rois_dev, spatial_scale,
                      pooled_h,
                      pooled_w, pool_channel, 0, top, argmax, stream);
}

extern "C" int pcnn_roi_pool_fwd_accumulate(const float* data, int B, int H, int W, int C, int layout,
                                            const float* rois, int R_cap, int roi_stride, int batch_base,
                                            const int32_t* num_rois_dev, float spatial_scale, int pooled_h,
                                            int pooled_w, int pool_channel, float* top, int32_t* argmax,
                                            void* stream) {
  return roi_pool_fwd(data, B, H, W, C, layout, rois, R_cap, roi_stride, batch_base, num_rois_dev, spatial_scale,
                      pooled_h,
                      pooled_w, pool_channel, 1, top, argmax, stream);
}

static int roi_pool_fwd_pair(const float* data_a, int Ha, int Wa, float scale_a, const float* data_b, int Hb, int Wb,
                             float scale_b, int B, int C, const float* rois, int R_cap, int roi_stride, int batch_base,
                             const int32_t* num_rois_dev, int pooled_h, int pooled_w, float* top_sum, void* argmax_a,
                             void* argmax_b, bool px, void* stream) {
  PCNN_REQUIRE(data_a && data_b && rois && top_sum && argmax_a && argmax_b && B > 0 && C > 0 && C % 4 == 0);
  PCNN_REQUIRE(Ha > 0 && Wa > 0 && Hb > 0 && Wb > 0 && pooled_h > 0 && pooled_w > 0 && R_cap >= 0);
  PCNN_REQUIRE(roi_stride >= 5);
  PCNN_REQUIRE((long)Ha * Wa * C < (1l << 31) && (long)Hb * Wb * C < (1l << 31));
  PCNN_REQUIRE(!px || ((long)Ha * Wa < 0xFFFF && (long)Hb * Wb < 0xFFFF));  // 0xFFFF marks an empty bin
  PCNN_REQUIRE(((((uintptr_t)data_a) | ((uintptr_t)data_b) | ((uintptr_t)top_sum)) & 15) == 0);
  PCNN_REQUIRE(((((uintptr_t)argmax_a) | ((uintptr_t)argmax_b)) & (px ? 7 : 15)) == 0);
  if (R_cap == 0) return PCNN_OK;
  const int threads = C / 4 >= 128 ? 128 : ((C / 4 + 63) / 64) * 64;
  if (px)
    hipLaunchKernelGGL(k_roi_fwd_pair_nhwc4<true>, dim3(fwd_grid(R_cap, pooled_h * pooled_w)), dim3(threads), 0,
                       (hipStream_t)stream, data_a, Ha, Wa, scale_a, data_b, Hb, Wb, scale_b, B, C, rois, R_cap,
                       roi_stride, batch_base, num_rois_dev, pooled_h, pooled_w, top_sum, argmax_a, argmax_b);
  else
    hipLaunchKernelGGL(k_roi_fwd_pair_nhwc4<false>, dim3(fwd_grid(R_cap, pooled_h * pooled_w)), dim3(threads), 0,
                       (hipStream_t)stream, data_a, Ha, Wa, scale_a, data_b, Hb, Wb, scale_b, B, C, rois, R_cap,
                       roi_stride, batch_base, num_rois_dev, pooled_h, pooled_w, top_sum, argmax_a, argmax_b);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_roi_pool_fwd_pair(const float* data_a, int Ha, int Wa, float scale_a, const float* data_b, int Hb,
                                      int Wb, float scale_b, int B, int C, const float* rois, int R_cap, int roi_stride,
                                      int batch_base, const int32_t* num_rois_dev, int pooled_h, int pooled_w, float* top_sum,
                                      int32_t* argmax_a, int32_t* argmax_b, void* stream) {
  return roi_pool_fwd_pair(data_a, Ha, Wa, scale_a, data_b, Hb, Wb, scale_b, B, C, rois, R_cap, roi_stride, batch_base,
                           num_rois_dev, pooled_h, pooled_w, top_sum, argmax_a, argmax_b, false, stream);
}

extern "C" int pcnn_roi_pool_fwd_pair_px(const float* data_a, int Ha, int Wa, float scale_a, const float* data_b,
                                         int Hb, int Wb, float scale_b, int B, int C, const float* rois, int R_cap,
                                         int roi_stride, int batch_base, const int32_t* num_rois_dev, int pooled_h,
                                         int pooled_w, float* top_sum, uint16_t* argmax_a, uint16_t* argmax_b,
                                         void* stream) {
  return roi_pool_fwd_pair(data_a, Ha, Wa, scale_a, data_b, Hb, Wb, scale_b, B, C, rois, R_cap, roi_stride, batch_base,
                           num_rois_dev, pooled_h, pooled_w, top_sum, argmax_a, argmax_b, true, stream);
}

extern "C" size_t pcnn_roi_pool_bwd_workspace_size(int B, int R_cap) {
  return pcnn::align_up((size_t)2 * (B > 0 ? B : 1) * sizeof(int32_t), 256) +
         pcnn::align_up((size_t)(R_cap > 0 ? R_cap : 1) * 8 * sizeof(int32_t), 256) + 256;
}

static int roi_pool_bwd(const float* top_diff, const void* argmax, bool px, int B, int H, int W, int C, int layout,
                        const float* rois, int R_cap, int roi_stride, int batch_base, const int32_t* num_rois_dev,
                        float spatial_scale, int pooled_h, int pooled_w, int pool_channel, float* bottom_diff,
                        void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(top_diff && argmax && rois && bottom_diff && workspace && B > 0 && H > 0 && W > 0 && C > 0);
  PCNN_REQUIRE(pooled_h > 0 && pooled_w > 0 && (layout == 0 || layout == 1) && R_cap >= 0);
  PCNN_REQUIRE(roi_stride >= 6 || (roi_stride == 5 && !pool_channel));
  PCNN_REQUIRE((long)H * W * C < (1l << 31));
  if (workspace_bytes < pcnn_roi_pool_bwd_workspace_size(B, R_cap)) return PCNN_ECAPACITY;
  hipStream_t st = (hipStream_t)stream;
  pcnn::Carve cv(workspace);
  int32_t* lo = cv.take<int32_t>(B);
  int32_t* hi = cv.take<int32_t>(B);
  int32_t* geo = cv.take<int32_t>((size_t)(R_cap > 0 ? R_cap : 1) * 8);
  hipLaunchKernelGGL(k_roi_prep, dim3(1), dim3(1024), 0, st, rois, R_cap, roi_stride, batch_base, num_rois_dev,
                     B, spatial_scale, pooled_h, pooled_w, geo, lo, hi);
  // tile shape: 2x4 pixels, or 1x4 when 2x4 tiles would leave the chip short
  // of workgroups (conv5_3 at 30x40: 4800 -> 9600 workgroups, measured
  // 64 -> 50 us; conv4_3 at 60x80 keeps 2x4: 77 vs 88 us for 1x4)
  const int nchunk = (C + kBChunk - 1) / kBChunk;
  const long wg24 = (long)B * ((H + 1) / 2) * ((W + 3) / 4) * nchunk;
  const bool narrow = wg24 < PCNN_RBW_NARROW;
#ifndef PCNN_RBW_TH
#define PCNN_RBW_TH 2
#endif
  const int tbh = narrow ? 1 : PCNN_RBW_TH, tbw = 4;
  const bool vec = layout == 0 && !pool_channel && C % 2 == 0 && pooled_h * tbh <= 32 && pooled_w * tbw <= 32 &&
                   (long)H * W * C < (1l << 30) && (long)R_cap * pooled_h * pooled_w * C < (1l << 29) &&
                   // top_diff is read as b64 and bottom_diff written as float2 in both forms;
                   // only the argmax (uint16 pixel indices in the px form) may be 4-byte aligned
                   (((uintptr_t)top_diff | (uintptr_t)bottom_diff) & 7) == 0 && ((uintptr_t)argmax & (px ? 3 : 7)) == 0;
  PCNN_REQUIRE(!px || (vec && (long)H * W < 0xFFFF));  // pixel-index argmax: the entry-list kernel only
  if (vec) {
    const int tiles = ((H + tbh - 1) / tbh) * ((W + tbw - 1) / tbw);
    const unsigned nwg = (unsigned)((B * tiles * nchunk + 7) / 8 * 8);
#define PCNN_RBW(TH, PXV)                                                                                  \
  pcnn::launch_last(k_roi_bwd_ent<TH, 4, PXV>, dim3(nwg), dim3(64 * kBWaves), 0, st, top_diff, argmax, B, H, W, C, \
                    geo, lo, hi, pooled_h, pooled_w, bottom_diff)
    if (narrow) {
      if (px) PCNN_RBW(1, true); else PCNN_RBW(1, false);
    } else {
      if (px) PCNN_RBW(PCNN_RBW_TH, true); else PCNN_RBW(PCNN_RBW_TH, false);
    }
#undef PCNN_RBW
  } else {
    if (hipMemsetAsync(bottom_diff, 0, (size_t)B * H * W * C * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
    const long npix = (long)B * H * W;
    const int blocks = (int)((npix + 255) / 256 < 8192 ? (npix + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_bwd_generic, dim3(blocks), dim3(256), 0, st, top_diff, (const int32_t*)argmax, B, H, W,
                       C, layout, geo, pooled_h, pooled_w, pool_channel, lo, hi, bottom_diff);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_roi_pool_bwd(const float* top_diff, const int32_t* argmax, int B, int H, int W, int C, int layout,
                                 const float* rois, int R_cap, int roi_stride, int batch_base,
                                 const int32_t* num_rois_dev, float spatial_scale, int pooled_h, int pooled_w,
                                 int pool_channel, float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
  return roi_pool_bwd(top_diff, argmax, false, B, H, W, C, layout, rois, R_cap, roi_stride, batch_base, num_rois_dev,
                      spatial_scale, pooled_h, pooled_w, pool_channel, bottom_diff, workspace, workspace_bytes, stream);
}

extern "C" int pcnn_roi_pool_bwd_px(const float* top_diff, const uint16_t* argmax_px, int B, int H, int W, int C,
                                    const float* rois, int R_cap, int roi_stride, int batch_base,
                                    const int32_t* num_rois_dev, float spatial_scale, int pooled_h, int pooled_w,
                                    float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
  return roi_pool_bwd(top_diff, argmax_px, true, B, H, W, C, 0, rois, R_cap, roi_stride, batch_base, num_rois_dev,
                      spatial_scale, pooled_h, pooled_w, 0, bottom_diff, workspace, workspace_bytes, stream);
}
