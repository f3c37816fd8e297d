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
// computed once (k_roi_prep); each workgroup owns a 4x8 pixel tile of one
// image, stages the (ordered) list of RoIs that intersect the tile in LDS, and
// one wave per pixel accumulates the argmax-matching top gradients of the 1-4
// bins containing it, in the reference's order (RoI ascending, ph, pw) — the
// fp32 sums are bit-equal to the reference kernel's.
#include "pcnn_common.h"
#include <math.h>
#include <cfloat>

namespace {

constexpr int kTileH = 2, kTileW = 4;
constexpr int kMaxTileRois = 1024;

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

// NHWC, all channels, C % 4 == 0: block (roi, bin), lane -> 4 channels.
// ACC: top += pooled (the pool5 + pool4 sum of vgg16_convs.py:184 produced in
// place by the second pool; the argmax of each map is still written).
template <bool ACC>
__global__ void __launch_bounds__(128) k_roi_fwd_nhwc4(const float* __restrict__ data, int B, int H, int W, int C,
                                                        const float* __restrict__ rois, int R_cap, int stride,
                                                        const int32_t* __restrict__ num_rois_dev, float scale, int PH,
                                                        int PW, float* __restrict__ top, int32_t* __restrict__ argmax) {
  const int r = blockIdx.x, bin = blockIdx.y;
  if (r >= rows_of(num_rois_dev, R_cap)) return;
  const int ph = bin / PW, pw = bin % PW;
  const RoiGeo g = roi_geo(rois, r, stride, scale, PH, PW);
  const bool bad = g.b < 0 || g.b >= B;
  int hs, he, ws, we;
  bin_bounds(g, ph, pw, H, W, hs, he, ws, we);
  const bool empty = bad || (he <= hs) || (we <= ws);
  const float* bd = data + (size_t)(bad ? 0 : g.b) * H * W * C;
  float* to = top + (((size_t)r * PH + ph) * PW + pw) * C;
  int32_t* ao = argmax + (((size_t)r * PH + ph) * PW + pw) * C;
  for (int c = threadIdx.x * 4; c < C; c += blockDim.x * 4) {
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
          upd(v0.x, i0 + 0, m0, a0); upd(v0.y, i0 + 1, m1, a1); upd(v0.z, i0 + 2, m2, a2); upd(v0.w, i0 + 3, m3, a3);
          upd(v1.x, i1 + 0, m0, a0); upd(v1.y, i1 + 1, m1, a1); upd(v1.z, i1 + 2, m2, a2); upd(v1.w, i1 + 3, m3, a3);
        }
        if (w < we) {
          const int i0 = (h * W + w) * C + c;
          const float4 v0 = *(const float4*)(bd + i0);
          upd(v0.x, i0 + 0, m0, a0); upd(v0.y, i0 + 1, m1, a1); upd(v0.z, i0 + 2, m2, a2); upd(v0.w, i0 + 3, m3, a3);
        }
      }
    }
    if (ACC) {
      const float4 p = *(const float4*)(to + c);
      *(float4*)(to + c) = make_float4(p.x + m0, p.y + m1, p.z + m2, p.w + m3);
    } else {
      *(float4*)(to + c) = make_float4(m0, m1, m2, m3);
    }
    *(int4*)(ao + c) = make_int4(a0, a1, a2, a3);
  }
}

// generic: one thread per output element (NCHW layout, pool_channel, C % 4 != 0)
__global__ void k_roi_fwd_generic(const float* __restrict__ data, int B, int H, int W, int C, int layout,
                                  const float* __restrict__ rois, int R_cap, int stride,
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
    top[idx] = acc ? top[idx] + maxval : maxval;
    argmax[idx] = maxidx;
  }
}

// RoI geometry once per row + per-image RoI index ranges.
// geo[r] = {b, cls, sw, sh, ew, eh, bits(bin_h), bits(bin_w)}
__global__ void __launch_bounds__(1024) k_roi_prep(const float* __restrict__ rois, int R_cap, int stride,
                                                    const int32_t* __restrict__ num_rois_dev, int B, float scale,
                                                    int PH, int PW, int32_t* __restrict__ geo,
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
    const RoiGeo g = roi_geo(rois, r, stride, scale, PH, PW);
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

// NHWC all-channel backward, C % 4 == 0: block = kTileH x kTileW pixel tile of
// one image.  The RoIs touching the tile are compacted (in order) into LDS;
// then one wave per pixel (1) tests the listed RoIs in parallel across lanes,
// (2) expands the containing RoIs, in order, into their (ph, pw) bins — the
// reference's summation order — as a wave-private entry list, and (3) issues
// the argmax / top-gradient loads of kBatch entries at a time before
// accumulating them in order (memory-level parallelism instead of one
// dependent round trip per bin).
constexpr int kEntCap = 64;
constexpr int kBatch = 4;

__global__ void __launch_bounds__(256) k_roi_bwd_tile(const float* __restrict__ top_diff,
                                                       const int32_t* __restrict__ argmax, int B, int H, int W, int C,
                                                       const int32_t* __restrict__ geo, const int32_t* __restrict__ lo,
                                                       const int32_t* __restrict__ hi, int PH, int PW,
                                                       float* __restrict__ bottom) {
  __shared__ int lst[kMaxTileRois];
  __shared__ int4 lgeo[kMaxTileRois];    // sw, sh, ew, eh of listed RoIs
  __shared__ float2 lbin[kMaxTileRois];  // bin_h, bin_w
  __shared__ int ent[4][kEntCap];        // per wave: element offsets ((r*PH+ph)*PW+pw)*C
  __shared__ int wcnt[4];
  __shared__ int nlist;
  const int tiles_w = (W + kTileW - 1) / kTileW, tiles_h = (H + kTileH - 1) / kTileH;
  const int b = blockIdx.x / (tiles_w * tiles_h);
  const int t = blockIdx.x % (tiles_w * tiles_h);
  const int h0 = (t / tiles_w) * kTileH, w0 = (t % tiles_w) * kTileW;
  const int h1 = min(h0 + kTileH, H) - 1, w1 = min(w0 + kTileW, W) - 1;
  const int lane = pcnn::lane_id(), wave = threadIdx.x >> 6;
  const int r0 = lo[b], r1 = hi[b];
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  for (int base = r0; base <= r1; base += blockDim.x) {  // ordered compaction
    const int r = base + threadIdx.x;
    bool hit = false;
    if (r <= r1) {
      const int32_t* g = geo + (size_t)r * 8;
      hit = g[0] == b && g[3] <= h1 && g[5] >= h0 && g[2] <= w1 && g[4] >= w0;
    }
    const uint64_t m = __ballot(hit);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int off = nlist;
    for (int w = 0; w < wave; w++) off += wcnt[w];
    if (hit) {
      const int pos = off + __popcll(m & pcnn::lanemask_lt());
      if (pos < kMaxTileRois) {
        const int32_t* g = geo + (size_t)r * 8;
        lst[pos] = r;
        lgeo[pos] = make_int4(g[2], g[3], g[4], g[5]);
        lbin[pos] = make_float2(__int_as_float(g[6]), __int_as_float(g[7]));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) nlist += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
  const int n = nlist;
  const bool use_list = n <= kMaxTileRois;  // else scan the image's RoI range (same order)
  const int nscan = use_list ? n : (r1 - r0 + 1);
  int* my = ent[wave];
  for (int p = wave; p < kTileH * kTileW; p += 4) {
    const int h = h0 + p / kTileW, w = w0 + p % kTileW;
    if (h >= H || w >= W) continue;
    const int pix = (h * W + w) * C;
    float* dst = bottom + ((size_t)b * H * W) * C + pix;
    for (int c0 = 0; c0 < C; c0 += 512) {
      const int ca = c0 + lane * 4, cb = c0 + 256 + lane * 4;
      const bool va = ca < C, vb = cb < C;
      float4 accA = make_float4(0.f, 0.f, 0.f, 0.f), accB = accA;
      int ne = 0;
      auto flush = [&]() {
        for (int e0 = 0; e0 < ne; e0 += kBatch) {
          int4 aa[kBatch], ab[kBatch];
          float4 da[kBatch], db[kBatch];
#pragma unroll
          for (int k = 0; k < kBatch; k++) {
            const int o = my[min(e0 + k, ne - 1)];
            aa[k] = va ? *(const int4*)(argmax + o + ca) : make_int4(-1, -1, -1, -1);
            da[k] = va ? *(const float4*)(top_diff + o + ca) : make_float4(0.f, 0.f, 0.f, 0.f);
            ab[k] = vb ? *(const int4*)(argmax + o + cb) : make_int4(-1, -1, -1, -1);
            db[k] = vb ? *(const float4*)(top_diff + o + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int k = 0; k < kBatch; k++) {
            if (e0 + k >= ne) break;
            const int ia = pix + ca, ib = pix + cb;
            if (aa[k].x == ia + 0) accA.x += da[k].x;
            if (aa[k].y == ia + 1) accA.y += da[k].y;
            if (aa[k].z == ia + 2) accA.z += da[k].z;
            if (aa[k].w == ia + 3) accA.w += da[k].w;
            if (ab[k].x == ib + 0) accB.x += db[k].x;
            if (ab[k].y == ib + 1) accB.y += db[k].y;
            if (ab[k].z == ib + 2) accB.z += db[k].z;
            if (ab[k].w == ib + 3) accB.w += db[k].w;
          }
        }
        ne = 0;
      };
      for (int l0 = 0; l0 < nscan; l0 += 64) {
        // lanes test 64 listed RoIs at once (cu.cc:172-177)
        const int li = l0 + lane;
        bool in = false;
        if (li < nscan) {
          int4 g;
          if (use_list) {
            g = lgeo[li];
          } else {
            const int32_t* gg = geo + (size_t)(r0 + li) * 8;
            g = gg[0] == b ? make_int4(gg[2], gg[3], gg[4], gg[5]) : make_int4(1, 1, 0, 0);
          }
          in = w >= g.x && w <= g.z && h >= g.y && h <= g.w;
        }
        uint64_t m = __ballot(in);
        while (m) {  // containing RoIs in order
          const int i = l0 + __ffsll((long long)m) - 1;
          m &= m - 1;
          const int r = use_list ? lst[i] : r0 + i;
          RoiGeo g;
          if (use_list) {
            const int4 q = lgeo[i];
            const float2 bn = lbin[i];
            g.sw = q.x; g.sh = q.y; g.ew = q.z; g.eh = q.w; g.bin_h = bn.x; g.bin_w = bn.y;
          } else {
            const int32_t* gg = geo + (size_t)r * 8;
            g.sw = gg[2]; g.sh = gg[3]; g.ew = gg[4]; g.eh = gg[5];
            g.bin_h = __int_as_float(gg[6]);
            g.bin_w = __int_as_float(gg[7]);
          }
          int phs, phe, pws, pwe;
          bins_of_pixel(g, h, w, PH, PW, phs, phe, pws, pwe);
          for (int ph = phs; ph < phe; ph++)
            for (int pw = pws; pw < pwe; pw++) {
              if (ne == kEntCap) flush();
              if (lane == 0) my[ne] = ((r * PH + ph) * PW + pw) * C;
              ne++;
            }
        }
      }
      flush();
      if (va) *(float4*)(dst + ca) = accA;
      if (vb) *(float4*)(dst + cb) = accB;
    }
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
                        int roi_stride, const int32_t* num_rois_dev, float spatial_scale, int pooled_h, int pooled_w,
                        int pool_channel, int acc, float* top, int32_t* argmax, void* stream) {
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
      hipLaunchKernelGGL(k_roi_fwd_nhwc4<true>, dim3(R_cap, pooled_h * pooled_w), dim3(threads), 0, st, data, B, H,
                         W, C, rois, R_cap, roi_stride, num_rois_dev, spatial_scale, pooled_h, pooled_w, top, argmax);
    else
      hipLaunchKernelGGL(k_roi_fwd_nhwc4<false>, dim3(R_cap, pooled_h * pooled_w), dim3(threads), 0, st, data, B, H,
                         W, C, rois, R_cap, roi_stride, num_rois_dev, spatial_scale, pooled_h, pooled_w, top, argmax);
  } else {
    const long n = (long)R_cap * pooled_h * pooled_w * (pool_channel ? 1 : C);
    const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_fwd_generic, dim3(blocks), dim3(256), 0, st, data, B, H, W, C, layout, rois, R_cap,
                       roi_stride, num_rois_dev, spatial_scale, pooled_h, pooled_w, pool_channel, acc, top, argmax);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_roi_pool_fwd(const float* data, int B, int H, int W, int C, int layout, const float* rois,
                                 int R_cap, int roi_stride, const int32_t* num_rois_dev, float spatial_scale,
                                 int pooled_h, int pooled_w, int pool_channel, float* top, int32_t* argmax,
                                 void* stream) {
  return roi_pool_fwd(data, B, H, W, C, layout, rois, R_cap, roi_stride, num_rois_dev, spatial_scale, pooled_h,
                      pooled_w, pool_channel, 0, top, argmax, stream);
}

extern "C" int pcnn_roi_pool_fwd_accumulate(const float* data, int B, int H, int W, int C, int layout,
                                            const float* rois, int R_cap, int roi_stride,
                                            const int32_t* num_rois_dev, float spatial_scale, int pooled_h,
                                            int pooled_w, int pool_channel, float* top, int32_t* argmax,
                                            void* stream) {
  return roi_pool_fwd(data, B, H, W, C, layout, rois, R_cap, roi_stride, num_rois_dev, spatial_scale, pooled_h,
                      pooled_w, pool_channel, 1, top, argmax, stream);
}

extern "C" size_t pcnn_roi_pool_bwd_workspace_size(int B, int R_cap) {
  return pcnn::align_up((size_t)2 * (B > 0 ? B : 1) * sizeof(int32_t), 256) +
         pcnn::align_up((size_t)(R_cap > 0 ? R_cap : 1) * 8 * sizeof(int32_t), 256) + 256;
}

extern "C" int pcnn_roi_pool_bwd(const float* top_diff, const int32_t* argmax, int B, int H, int W, int C, int layout,
                                 const float* rois, int R_cap, int roi_stride, const int32_t* num_rois_dev,
                                 float spatial_scale, int pooled_h, int pooled_w, int pool_channel,
                                 float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream) {
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
  hipLaunchKernelGGL(k_roi_prep, dim3(1), dim3(1024), 0, st, rois, R_cap, roi_stride, num_rois_dev, B,
                     spatial_scale, pooled_h, pooled_w, geo, lo, hi);
  const bool vec = layout == 0 && !pool_channel && C % 4 == 0 && C <= 4096 &&
                   (((uintptr_t)top_diff | (uintptr_t)argmax | (uintptr_t)bottom_diff) & 15) == 0;
  if (vec) {
    const int tiles = ((H + kTileH - 1) / kTileH) * ((W + kTileW - 1) / kTileW);
    hipLaunchKernelGGL(k_roi_bwd_tile, dim3(B * tiles), dim3(256), 0, st, top_diff, argmax, B, H, W, C, geo, lo, hi,
                       pooled_h, pooled_w, bottom_diff);
  } else {
    if (hipMemsetAsync(bottom_diff, 0, (size_t)B * H * W * C * sizeof(float), st) != hipSuccess) return PCNN_EHIP;
    const long npix = (long)B * H * W;
    const int blocks = (int)((npix + 255) / 256 < 8192 ? (npix + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_roi_bwd_generic, dim3(blocks), dim3(256), 0, st, top_diff, argmax, B, H, W, C, layout, geo,
                       pooled_h, pooled_w, pool_channel, lo, hi, bottom_diff);
  }
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
