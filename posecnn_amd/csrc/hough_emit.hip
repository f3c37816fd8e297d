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
#include <algorithm>
#include <cmath>

namespace pcnn_hough {

constexpr int kEmitMax = 256;  // maxima per image (>= pks)

// One workgroup per image: per-max geometry first (box, GT match), then the
// image's rows written by all threads (coalesced target / weight rows).
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
  __shared__ float s_box[kEmitMax][4];
  __shared__ float s_pose[kEmitMax][3];
  __shared__ float s_score[kEmitMax];
  __shared__ int s_cls[kEmitMax], s_gsel[kEmitMax];
  __shared__ int s_off, s_total;
  const int b = blockIdx.x;
  const int rpm = is_train ? 9 : 1;
  const int PC = 4 * C;
  if (threadIdx.x == 0) {
    int off = 0, tot = 0;
    for (int i = 0; i < B; i++) {
      if (i == b) off = tot;
      tot += ws.nvote[i] * rpm;
    }
    s_off = off;
    s_total = tot;
  }
  const int nk = min(ws.nvote[b], kEmitMax);
  const float* mb = meta + (size_t)b * num_meta;
  const int batch_index = batch_base + b;
  for (int k = threadIdx.x; k < nk; k += blockDim.x) {
    const float* pk = ws.peak + ((size_t)b * ws.pks + k) * 8;
    const int slot = nms ? (int)pk[6] : k;
    const int cls = ws.slot_cls[(size_t)b * C + slot];
    const float bb_distance = pk[1], bb_height = pk[2], bb_width = pk[3];
    const int x = (int)pk[4], y = (int)pk[5];
    const float fx = mb[0], fy = mb[4], px = mb[2], py = mb[5];
    const float rx = ((float)x - px) / fx;  // cu.cc:404-405
    const float ry = ((float)y - py) / fy;
    const double sc = 0.5 + (double)0.05f;  // x - bb_width * (0.5 + scale), evaluated in double (cu.cc:417-420)
    float bx[4];
    bx[0] = (float)((double)x - (double)bb_width * sc);
    bx[1] = (float)((double)y - (double)bb_height * sc);
    bx[2] = (float)((double)x + (double)bb_width * sc);
    bx[3] = (float)((double)y + (double)bb_height * sc);
    int gsel = -1;
    if (is_train) {  // first same-(b, cls) GT whose projected box overlaps > 0.2 (cu.cc:440-466)
      for (int i = 0; i < num_gt; i++) {
        const int gt_batch = (int)gt[i * 13 + 0];
        const int gt_id = (int)gt[i * 13 + 1];
        if (cls == gt_id && batch_index == gt_batch) {
          const float ov = box_overlap(cls, extents, mb, gt + (size_t)i * 13, bx);
          if ((double)ov > 0.2) {
            gsel = i;
            break;
          }
        }
      }
    }
    for (int t = 0; t < 4; t++) s_box[k][t] = bx[t];
    s_pose[k][0] = rx * bb_distance;
    s_pose[k][1] = ry * bb_distance;
    s_pose[k][2] = bb_distance;
    s_score[k] = pk[0];
    s_cls[k] = cls;
    s_gsel[k] = gsel;
  }
  __syncthreads();
  const int off = s_off, total = s_total;
  const int nrows = nk * rpm;
  // jitter order of cu.cc:476-554: (0,0) then (-,-) (+,-) (-,+) (+,+) (0,-) (-,0) (0,+) (+,0)
  const int jx[9] = {0, -1, 1, -1, 1, 0, -1, 0, 1};
  const int jy[9] = {0, -1, -1, 1, 1, -1, 0, 1, 0};
  for (int i = threadIdx.x; i < nrows; i += blockDim.x) {
    const int k = i / rpm, j = i % rpm;
    const int r = off + i;
    if (r >= cap) {
      atomicAdd(&ws.diag[2], 1);
      continue;
    }
    float* bo = top_box + (size_t)r * 7;
    const float x1 = s_box[k][0], y1 = s_box[k][1];
    bo[0] = (float)batch_index;
    bo[1] = (float)s_cls[k];
    if (j == 0) {
      bo[2] = x1; bo[3] = y1; bo[4] = s_box[k][2]; bo[5] = s_box[k][3];
    } else {
      const float ww = s_box[k][2] - x1, hh = s_box[k][3] - y1;
      const float nx = jx[j] == 0 ? x1 : (float)((double)x1 + (jx[j] < 0 ? -0.05 : 0.05) * (double)ww);
      const float ny = jy[j] == 0 ? y1 : (float)((double)y1 + (jy[j] < 0 ? -0.05 : 0.05) * (double)hh);
      bo[2] = nx;
      bo[3] = ny;
      bo[4] = nx + ww;
      bo[5] = ny + hh;
    }
    bo[6] = s_score[k];
    float* po = top_pose + (size_t)r * 7;
    po[0] = 1.f; po[1] = 0.f; po[2] = 0.f; po[3] = 0.f;
    po[4] = s_pose[k][0];
    po[5] = s_pose[k][1];
    po[6] = s_pose[k][2];
    top_domain[r] = is_train ? (num_gt == 0 ? 1 : 0) : 0;
  }
  const long ncol = (long)nrows * PC;
  for (long idx = threadIdx.x; idx < ncol; idx += blockDim.x) {
    const int i = (int)(idx / PC), col = (int)(idx % PC);
    const int r = off + i;
    if (r >= cap) continue;
    const int k = i / rpm;
    const int g = s_gsel[k], cls = s_cls[k];
    const bool on = g >= 0 && col >= 4 * cls && col < 4 * cls + 4;
    top_target[(size_t)r * PC + col] = on ? gt[g * 13 + 6 + (col - 4 * cls)] : 0.f;
    top_weight[(size_t)r * PC + col] = on ? 1.f : 0.f;
  }
  if (b == 0) {
    if (threadIdx.x == 0) {
      const int n = total < cap ? total : cap;
      num_rois[0] = n;
      num_rois[1] = n > 0 ? n : 1;
    }
    if (total == 0) {  // dummy all-zero row (hough_voting_gpu_op.cc:382-383)
      for (int t = threadIdx.x; t < 7; t += blockDim.x) {
        top_box[t] = 0.f;
        top_pose[t] = 0.f;
      }
      for (int t = threadIdx.x; t < PC; t += blockDim.x) {
        top_target[t] = 0.f;
        top_weight[t] = 0.f;
      }
      if (threadIdx.x == 0) top_domain[0] = 0;
    }
  }
}

}  // namespace pcnn_hough

using namespace pcnn_hough;

extern "C" size_t pcnn_hough_voting_workspace_size(int B, int H, int W, int C, int skip_pixels, float vote_thr) {
  if (B <= 0 || H <= 0 || W <= 0 || C < 2 || skip_pixels <= 0) return 0;
  size_t bytes = 0;
  carve_ws(nullptr, B, H, W, C, skip_pixels, vote_thr > 0.f, &bytes);
  return bytes + 256;
}

extern "C" int pcnn_hough_voting(const int32_t* label, const float* vertex, const float* extents, const float* meta,
                                 int num_meta, const float* gt, int num_gt, int B, int H, int W, int C,
                                 int batch_base, int global_batch, int is_train, float inlier_thr, int label_thr,
                                 float vote_thr, float per_thr, int skip_pixels, float* top_box, float* top_pose,
                                 float* top_target, float* top_weight, int32_t* top_domain, int32_t* num_rois,
                                 int cap, int32_t* debug_counts, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && C >= 2 && C <= kMaxClasses && skip_pixels > 0 && num_meta >= 6);
  PCNN_REQUIRE((long)H * W * (C - 1) < (1l << 31) && W < (1 << 16));
  PCNN_REQUIRE(label && vertex && extents && meta && top_box && top_pose && top_target && top_weight &&
               top_domain && num_rois && workspace && cap > 0);
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

  if (hipMemsetAsync(ws.diag, 0, 4 * sizeof(int32_t), st) != hipSuccess) return PCNN_EHIP;
  hipLaunchKernelGGL(k_label_hist, dim3(ws.nblk, B), dim3(kCompactThreads), 0, st, label, HW, C, ws);
  hipLaunchKernelGGL(k_label_scan, dim3(B), dim3(1024), 0, st, C, label_thr, index_size, nms ? 1 : 0, skip_pixels,
                     ws);
  hipLaunchKernelGGL(k_label_scatter, dim3(ws.nblk, B), dim3(kCompactThreads), 0, st, label, vertex, extents, meta,
                     num_meta, H, W, C, skip_pixels, ws);
  {
    const double c = (double)inlier_thr, co = c - kConeEps, ci = c + kConeEps;
    const double so = std::sqrt(std::max(0.0, 1.0 - co * co)), si = std::sqrt(std::max(0.0, 1.0 - ci * ci));
    hipLaunchKernelGGL(k_voter_setup, dim3((ws.vcap + 255) / 256, B), dim3(256), 0, st, inlier_thr, so, si, ws);
  }
  PCNN_CHECK_LAUNCH();
  int32_t* counts_out = nms ? ws.counts : debug_counts;
  // slots that can vote: all present classes (NMS) or the first index_size (cu.cc:775-776)
  const int slots = nms ? C - 1 : (C - 1 < index_size ? C - 1 : index_size);
  if (slots > 0) {
    const size_t lds = (size_t)kBand * (W + 1) * sizeof(int);
    hipLaunchKernelGGL(k_hough_vote, dim3((H + kBand - 1) / kBand, slots, B), dim3(kVoteThreads), lds, st, H, W, C,
                       inlier_thr, ws, counts_out);
    PCNN_CHECK_LAUNCH();
    if (!nms) {
      hipLaunchKernelGGL(k_hough_peak, dim3(slots, B), dim3(kPeakThreads), 0, st, H, W, C, inlier_thr, extents,
                         meta, num_meta, ws);
    } else {
      hipLaunchKernelGGL(k_hough_nms_cand, dim3((HW + 255) / 256 < 64 ? (HW + 255) / 256 : 64, C - 1, B),
                         dim3(256), 0, st, H, W, C, vote_thr, ws);
      hipLaunchKernelGGL(k_hough_cand_data, dim3(128, B), dim3(kPeakThreads), 0, st, H, W, C, inlier_thr, extents,
                         meta, num_meta, ws);
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
  hipLaunchKernelGGL(k_hough_emit, dim3(B), dim3(kEmitThreads), 0, st, B, H, W, C, is_train, batch_base,
                     nms ? 1 : 0, extents, meta, num_meta, gt, num_gt, ws, top_box, top_pose, top_target,
                     top_weight, top_domain, num_rois, cap);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
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
