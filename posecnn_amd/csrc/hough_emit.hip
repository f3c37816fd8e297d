// Hough voting for PoseCNN on MI355X (gfx950): RoI emission and the C-ABI.
//
// Replaces HoughVotingLaucher (lib/hough_voting_gpu_layer/hough_voting_gpu_op.cu.cc:615-799)
// and the per-image loop of HoughvotinggpuOp<GPU>::Compute (hough_voting_gpu_op.cc:321-429).
// The reference does count * H * W * N_c / skip predicate evaluations per
// image with ~6 host syncs; this op produces the same outputs (canonical
// order) with no host synchronisation:
//   hough_compact.hip  voter lists in ascending raster order (cu.cc:174-187, :644-678)
//   hough_vote.hip     interval vote -> per-class first maximum (cu.cc:253-294, :757)
//   hough_peak.hip     exact hough_data at maxima / NMS candidates (cu.cc:296-383)
//   this file          compute_rois_kernel (cu.cc:386-576): image-major rows,
//                      ascending slot / flat order, capacity-sized outputs and a
//                      device-side row count (+ dummy row, hough_voting_gpu_op.cc:382-383)
#include "hough_common.h"
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <cmath>

namespace pcnn_hough {

// Multi-instance (NMS) path and the no-slot case: one workgroup per image,
// its kept maxima in selection order (ascending flat (slot, y, x), cu.cc:351-380).
__global__ void __launch_bounds__(kEmitThreads) k_hough_emit(int B, int H, int W, int C, int is_train,
                                                              int batch_base, int nms,
                                                              const float* __restrict__ extents,
                                                              const float* __restrict__ meta, int num_meta,
                                                              const float* __restrict__ gt, int num_gt, HoughWs ws,
                                                              float* __restrict__ top_box,
                                                              float* __restrict__ top_pose,
                                                              float* __restrict__ top_target,
                                                              float* __restrict__ top_weight,
                                                              int32_t* __restrict__ top_domain,
                                                              int32_t* __restrict__ num_rois, int cap) {
  __shared__ EmitShared esh;
  __shared__ int s_off, s_total;
  const int b = blockIdx.x;
  const int rpm = is_train ? 9 : 1;
  if (threadIdx.x == 0) {
    int off = 0, tot = 0;
    for (int i = 0; i < B; i++) {
      if (i == b) off = tot;
      tot += ws.nvote[i] * rpm;
    }
    s_off = off;
    s_total = tot;
  }
  __syncthreads();
  const int nk = ws.nvote[b];
  const float* mb = meta + (size_t)b * num_meta;
  for (int k = 0; k < nk; k++) {
    const float* pk = ws.peak + ((size_t)b * ws.pks + k) * 8;
    const int slot = nms ? (int)pk[6] : k;
    const int cls = ws.slot_cls[(size_t)b * C + slot];
    emit_max(esh, s_off + k * rpm, cap, batch_base + b, cls, pk[0], pk[1], pk[2], pk[3], (int)pk[4], (int)pk[5],
             is_train, C, extents + (size_t)cls * 3, mb, gt, num_gt, top_box, top_pose, top_target, top_weight,
             top_domain, ws.diag);
    __syncthreads();
  }
  if (b == 0) emit_count(s_total, cap, C, top_box, top_pose, top_target, top_weight, top_domain, num_rois);
}

}  // namespace pcnn_hough

using namespace pcnn_hough;

extern "C" size_t pcnn_hough_voting_workspace_size(int B, int H, int W, int C, int skip_pixels, float vote_thr) {
  if (B <= 0 || H <= 0 || W <= 0 || C < 2 || skip_pixels <= 0) return 0;
  size_t bytes = 0;
  carve_ws(nullptr, B, H, W, C, skip_pixels, vote_thr > 0.f, &bytes);
  return bytes + 256;
}

// label given (pcnn_hough_voting) or produced from prob_normalized by the
// fused argmax (pcnn_hough_voting_prob: label = label_out, written here).
static int hough_voting_impl(const int32_t* label, const float* prob, int32_t* label_out, const float* vertex,
                             int vch, const float* extents, const float* meta, int num_meta, const float* gt, int num_gt,
                             int B, int H, int W, int C, int batch_base, int global_batch, int is_train,
                             float inlier_thr, int label_thr, float vote_thr, float per_thr, int skip_pixels,
                             float* top_box, float* top_pose, float* top_target, float* top_weight,
                             int32_t* top_domain, int32_t* num_rois, int cap, int32_t* debug_counts,
                             void* workspace, size_t workspace_bytes, void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C >= 2 && C <= kMaxClasses && skip_pixels > 0 && num_meta >= 6);
  PCNN_REQUIRE((long)H * W * (C - 1) < (1l << 31) && W < (1 << 16));
  PCNN_REQUIRE((label || (prob && label_out && (long)H * W * C < (1l << 31))) && vertex && extents && meta &&
               top_box && top_pose && top_target && top_weight && top_domain && num_rois && workspace && cap > 0);
  PCNN_REQUIRE(num_gt == 0 || gt);
  if (global_batch <= 0) global_batch = B;
  PCNN_REQUIRE(global_batch >= B);
  const bool nms = vote_thr > 0.f;
  size_t need = 0;
  carve_ws(nullptr, B, H, W, C, skip_pixels, nms, &need);
  if (workspace_bytes < need) return PCNN_ECAPACITY;
  HoughWs ws = carve_ws(workspace, B, H, W, C, skip_pixels, nms, nullptr);
  hipStream_t st = (hipStream_t)stream;
  const int index_size = PCNN_MAX_ROI / global_batch;  // cu.cc:734
  const int HW = H * W;
  // Sigma d at the maxima (hough_peak.hip): the in-order fp32 sum rebuilt in
  // parallel (default), or the one-lane serial chain everywhere when the
  // environment sets PCNN_HOUGH_SUM=serial (a test / A-B knob; both give the
  // same bits)
  const char* sum_mode = getenv("PCNN_HOUGH_SUM");
  const int psum = (sum_mode && strcmp(sum_mode, "serial") == 0) ? 0 : 1;

  if (label) {
    hipLaunchKernelGGL(k_label_hist, dim3(ws.nblk, B), dim3(kCompactThreads), 0, st, label, HW, C, H, ws);
  } else {
    const size_t lds = C <= kArgmaxStagedMaxC ? (size_t)kCompactThreads * C * sizeof(float) : 0;
    hipLaunchKernelGGL(k_label_hist_prob, dim3(ws.nblk, B), dim3(kCompactThreads), lds, st, prob, label_out, HW, C, H,
                       ws);
    label = label_out;
  }
  {
    const double c = (double)inlier_thr, co = c - kConeEps, ci = c + kConeEps;
    const double so = std::sqrt(std::max(0.0, 1.0 - co * co)), si = std::sqrt(std::max(0.0, 1.0 - ci * ci));
    // the placement's dynamic LDS grows with C and 1 / skip (57 KiB at C = 256,
    // skip = 1): above the 64 KiB default window (with the kernel's ~9 KiB of
    // static LDS) the launch needs the attribute raised, up to the CU's
    // 160 KiB (such launches used to fail)
    const size_t place_lds = place_lds_bytes(C, skip_pixels);
    if (place_lds + kPlaceStaticLds > 160 * 1024) return PCNN_ECAPACITY;
    if (place_lds + kPlaceStaticLds > 48 * 1024 &&
        hipFuncSetAttribute((const void*)k_label_place, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)place_lds) != hipSuccess)
      return PCNN_EHIP;
    hipLaunchKernelGGL(k_label_place, dim3(ws.nblk, B), dim3(kCompactThreads), place_lds, st,
                       label, vertex, vch, extents,
                       meta, num_meta, H, W, C, skip_pixels, label_thr, index_size, nms ? 1 : 0, inlier_thr, so, si,
                       ws);
  }
  PCNN_CHECK_LAUNCH();
  int32_t* counts_out = nms ? ws.counts : debug_counts;
  // slots that can vote: all present classes (NMS) or the first index_size (cu.cc:775-776)
  const int slots = nms ? C - 1 : (C - 1 < index_size ? C - 1 : index_size);
  if (slots > 0) {
    // vote geometry by batch (hough_vote.hip): two-row bands when B <= 2
    const int band = B <= 2 ? 2 : 4;
    const size_t lds = (size_t)band * (W + 1) * sizeof(int);
    const dim3 vgrid((H + band - 1) / band, slots, B);
    if (band == 4)
      hipLaunchKernelGGL((k_hough_vote<4, 512>), vgrid, dim3(512), lds, st, H, W, C, inlier_thr, ws, counts_out);
    else
      hipLaunchKernelGGL((k_hough_vote<2, 512>), vgrid, dim3(512), lds, st, H, W, C, inlier_thr, ws, counts_out);
    PCNN_CHECK_LAUNCH();
    if (!nms) {
      hipLaunchKernelGGL(k_hough_peak, dim3(slots, B), dim3(kPeakThreads), 0, st, B, H, W, C, inlier_thr, extents,
                         meta, num_meta, ws, is_train, batch_base, gt, num_gt, top_box, top_pose, top_target,
                         top_weight, top_domain, num_rois, cap, psum);
    } else {
      hipLaunchKernelGGL(k_hough_nms_cand, dim3((HW + 255) / 256 < 64 ? (HW + 255) / 256 : 64, C - 1, B),
                         dim3(256), 0, st, H, W, C, vote_thr, ws);
      hipLaunchKernelGGL(k_hough_cand_data, dim3(128, B), dim3(kPeakThreads), 0, st, H, W, C, inlier_thr, extents,
                         meta, num_meta, ws, psum);
      hipLaunchKernelGGL(k_hough_nms_select, dim3(B), dim3(1024), 0, st, H, W, C, per_thr, index_size, ws);
      if (debug_counts &&
          hipMemcpyAsync(debug_counts, ws.counts, (size_t)B * (C - 1) * HW * sizeof(int32_t),
                         hipMemcpyDeviceToDevice, st) != hipSuccess)
        return PCNN_EHIP;
    }
    PCNN_CHECK_LAUNCH();
  } else if (hipMemsetAsync(ws.nvote, 0, B * sizeof(int32_t), st) != hipSuccess) {
    return PCNN_EHIP;
  }
  if (nms || slots <= 0)  // the default path emits its rows in k_hough_peak
    hipLaunchKernelGGL(k_hough_emit, dim3(B), dim3(kEmitThreads), 0, st, B, H, W, C, is_train, batch_base,
                       nms ? 1 : 0, extents, meta, num_meta, gt, num_gt, ws, top_box, top_pose, top_target,
                       top_weight, top_domain, num_rois, cap);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hough_voting(const int32_t* label, const float* vertex, const float* extents, const float* meta,
                                 int num_meta, const float* gt, int num_gt, int B, int H, int W, int C,
                                 int batch_base, int global_batch, int is_train, float inlier_thr, int label_thr,
                                 float vote_thr, float per_thr, int skip_pixels, float* top_box, float* top_pose,
                                 float* top_target, float* top_weight, int32_t* top_domain, int32_t* num_rois,
                                 int cap, int32_t* debug_counts, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  if (!label) return PCNN_EINVAL;
  return hough_voting_impl(label, nullptr, nullptr, vertex, 3 * C, extents, meta, num_meta, gt, num_gt, B, H, W, C,
                           batch_base, global_batch, is_train, inlier_thr, label_thr, vote_thr, per_thr, skip_pixels,
                           top_box, top_pose, top_target, top_weight, top_domain, num_rois, cap, debug_counts,
                           workspace, workspace_bytes, stream);
}

extern "C" int pcnn_hough_voting_prob(const float* prob, int32_t* label_out, const float* vertex,
                                      const float* extents, const float* meta, int num_meta, const float* gt,
                                      int num_gt, int B, int H, int W, int C, int batch_base, int global_batch,
                                      int is_train, float inlier_thr, int label_thr, float vote_thr, float per_thr,
                                      int skip_pixels, float* top_box, float* top_pose, float* top_target,
                                      float* top_weight, int32_t* top_domain, int32_t* num_rois, int cap,
                                      int32_t* debug_counts, void* workspace, size_t workspace_bytes,
                                      void* stream) {
  if (!prob || !label_out) return PCNN_EINVAL;
  return hough_voting_impl(nullptr, prob, label_out, vertex, 3 * C, extents, meta, num_meta, gt, num_gt, B, H, W, C,
                           batch_base, global_batch, is_train, inlier_thr, label_thr, vote_thr, per_thr, skip_pixels,
                           top_box, top_pose, top_target, top_weight, top_domain, num_rois, cap, debug_counts,
                           workspace, workspace_bytes, stream);
}

extern "C" int pcnn_hough_voting_compact(const int32_t* label, const float* vertex3, const float* extents,
                                         const float* meta, int num_meta, const float* gt, int num_gt, int B, int H,
                                         int W, int C, int batch_base, int global_batch, int is_train,
                                         float inlier_thr, int label_thr, float vote_thr, float per_thr,
                                         int skip_pixels, float* top_box, float* top_pose, float* top_target,
                                         float* top_weight, int32_t* top_domain, int32_t* num_rois, int cap,
                                         int32_t* debug_counts, void* workspace, size_t workspace_bytes,
                                         void* stream) {
  if (!label) return PCNN_EINVAL;
  return hough_voting_impl(label, nullptr, nullptr, vertex3, 3, extents, meta, num_meta, gt, num_gt, B, H, W, C,
                           batch_base, global_batch, is_train, inlier_thr, label_thr, vote_thr, per_thr, skip_pixels,
                           top_box, top_pose, top_target, top_weight, top_domain, num_rois, cap, debug_counts,
                           workspace, workspace_bytes, stream);
}

extern "C" int pcnn_hough_voting_grad(float* grad_label, float* grad_vertex, int B, int H, int W, int C,
                                      void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0);
  hipStream_t st = (hipStream_t)stream;
  if (grad_label && hipMemsetAsync(grad_label, 0, (size_t)B * H * W * sizeof(float), st) != hipSuccess)
    return PCNN_EHIP;
  if (grad_vertex && hipMemsetAsync(grad_vertex, 0, (size_t)B * H * W * 3 * C * sizeof(float), st) != hipSuccess)
    return PCNN_EHIP;
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_hough_voting_diag(const void* workspace, int B, int H, int W, int C, int skip_pixels,
                                      float vote_thr, int32_t* diag_host4, void* stream) {
  PCNN_REQUIRE(workspace && diag_host4);
  HoughWs ws = carve_ws((void*)workspace, B, H, W, C, skip_pixels, vote_thr > 0.f, nullptr);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemcpyAsync(diag_host4, ws.diag, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
    return PCNN_EHIP;
  if (hipStreamSynchronize(st) != hipSuccess) return PCNN_EHIP;
  return PCNN_OK;
}
