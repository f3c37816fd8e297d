/*
 * posecnn_hip.h — C-ABI of libposecnn_hip.so, the MI355X (gfx950) replacement
 * for the native launchers behind PoseCNN's custom ops.
 *
 * Conventions
 *  - every pointer is a DEVICE pointer unless the name ends in _host;
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream);
 *  - nothing allocates: temporaries live in a caller-provided `workspace` whose
 *    size the matching *_workspace_size() query returns;
 *  - nothing synchronises: variable-length results (RoI rows) are written into
 *    capacity-sized buffers with a device-side row count, so a whole
 *    vote -> RoI pool -> FC -> loss step can be captured in a hipGraph;
 *  - return value 0 = PCNN_OK, otherwise a PCNN_E* code (never exit()).
 *
 * Reference seam replaced (mrlooi/PoseCNN): the TF OpKernel::Compute methods
 * call C++ launchers with raw device pointers + an Eigen::GpuDevice stream.
 */
#ifndef POSECNN_HIP_H
#define POSECNN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCNN_OK 0
#define PCNN_EINVAL 1    /* bad shape / argument (reference: OP_REQUIRES InvalidArgument) */
#define PCNN_EHIP 2      /* HIP launch error (reference: fprintf + exit(-1)) */
#define PCNN_ECAPACITY 3 /* workspace or output capacity too small */

#define PCNN_MAX_ROI 128 /* hough_voting_gpu_op.cu.cc:14 */

int pcnn_abi_version(void);
const char* pcnn_strerror(int code);

/* Completion event of the next op called on this thread (a created
 * hipEvent_t): the op's last kernel records it through the kernel's own
 * completion signal (hipExtLaunchKernel's stop event), so another stream can
 * be forked off at that point without an event-record marker on the op's
 * stream. Implemented by the fused ADD loss + head backward, the FC GEMMs
 * (precision 2) and the RoI-pool backward; after any other op the event stays
 * pending: pcnn_completion_event_pending() reports it (1) and clears it.
 * (No reference counterpart: a host-side scheduling hook of the pose step.) */
int pcnn_set_completion_event(void* event);
int pcnn_completion_event_pending(void);

/* ---------------------------------------------------------------------------
 * Hough voting (Houghvotinggpu).
 * Replaces HoughVotingLaucher (lib/hough_voting_gpu_layer/hough_voting_gpu_op.cu.cc:615-799)
 * called per image from HoughvotinggpuOp<GPU>::Compute (hough_voting_gpu_op.cc:321-429).
 *  label  (B,H,W) int32          vertex (B,H,W,3C) f32      extents (C,3) f32
 *  meta   (B,num_meta) f32       gt (num_gt,13) f32 [b,cls,0,0,0,0,qw,qx,qy,qz,tx,ty,tz]
 *  outputs, capacity `cap` rows (reference MAX_ROI*9 = 1152):
 *    top_box (cap,7) [b,cls,x1,y1,x2,y2,score]  top_pose (cap,7) [qw,qx,qy,qz,tx,ty,tz]
 *    top_target/top_weight (cap,4C)              top_domain (cap) int32
 *    num_rois (2) int32: [0] = rows emitted, [1] = max(rows, 1) (the op's
 *    output row count; row 0 is the all-zero dummy when rows == 0,
 *    hough_voting_gpu_op.cc:382-383)
 *  batch_base   added to the batch column (image-sharded runs, global image index)
 *  global_batch index_size = PCNN_MAX_ROI / global_batch (cu.cc:734)
 *  inlier_thr = 0.9, label_thr = 500 in the reference (hough_voting_gpu_op.cc:356-357)
 *  vote_thr <= 0: single instance per class (argmax); > 0: Hough-space NMS.
 *  debug_counts (optional, may be NULL): (B, C-1, H, W) int32 vote counts per
 *    present-class slot (slot order = ascending class id), the reference hough_space.
 * ------------------------------------------------------------------------- */
size_t pcnn_hough_voting_workspace_size(int B, int H, int W, int C, int skip_pixels, float vote_thr);

int pcnn_hough_voting(const int32_t* label, const float* vertex, const float* extents, const float* meta,
                      int num_meta, const float* gt, int num_gt, int B, int H, int W, int C, int batch_base,
                      int global_batch, int is_train, float inlier_thr, int label_thr, float vote_thr,
                      float per_thr, int skip_pixels, float* top_box, float* top_pose, float* top_target,
                      float* top_weight, int32_t* top_domain, int32_t* num_rois, int cap, int32_t* debug_counts,
                      void* workspace, size_t workspace_bytes, void* stream);

/* pcnn_hough_voting with the label producer fused in:
 * instead of label_2d the op takes prob_normalized (B,H,W,C) fp32 — the
 * softmax whose argmax is label_2d (argmax_2d, lib/networks/network.py:433-434;
 * graph vgg16_convs.py:144-146 -> :167-170) — labels every pixel inside the
 * compaction pass (first maximum; a NaN wins at its first occurrence, as
 * numpy / tf.argmax) and writes label_out (B,H,W) int32 as a by-product.
 * Outputs are those of pcnn_hough_voting on label_out; same workspace size. */
int pcnn_hough_voting_prob(const float* prob, int32_t* label_out, const float* vertex, const float* extents,
                           const float* meta, int num_meta, const float* gt, int num_gt, int B, int H, int W, int C,
                           int batch_base, int global_batch, int is_train, float inlier_thr, int label_thr,
                           float vote_thr, float per_thr, int skip_pixels, float* top_box, float* top_pose,
                           float* top_target, float* top_weight, int32_t* top_domain, int32_t* num_rois, int cap,
                           int32_t* debug_counts, void* workspace, size_t workspace_bytes, void* stream);

/* pcnn_hough_voting on a class-compact vertex map:
 * vertex3 (B,H,W,3) holds, per pixel, the 3 vertex channels of that pixel's
 * own label class (pcnn_vertex_pred_compact) instead of all 3C. Voters read
 * only their own class's channels (cu.cc:276-280), so the outputs equal
 * pcnn_hough_voting on any full map with those channels. C = num classes. */
int pcnn_hough_voting_compact(const int32_t* label, const float* vertex3, const float* extents, const float* meta,
                              int num_meta, const float* gt, int num_gt, int B, int H, int W, int C, int batch_base,
                              int global_batch, int is_train, float inlier_thr, int label_thr, float vote_thr,
                              float per_thr, int skip_pixels, float* top_box, float* top_pose, float* top_target,
                              float* top_weight, int32_t* top_domain, int32_t* num_rois, int cap,
                              int32_t* debug_counts, void* workspace, size_t workspace_bytes, void* stream);

/* HoughvotinggpuGrad (hough_voting_gpu_op.cc:440-484; set_gradients cu.cc:608-612):
 * zero gradients for label (B,H,W) and vertex (B,H,W,3C). Either may be NULL. */
int pcnn_hough_voting_grad(float* grad_label, float* grad_vertex, int B, int H, int W, int C, void* stream);

/* Diagnostic counters of the last pcnn_hough_voting call on `workspace`:
 * copies [0] = count mismatches between the interval vote and the exact
 * per-voter re-check at emitted maxima (must be 0), [1] = NMS candidate
 * overflows, [2] = RoI rows past the output capacity, [3] = maxima whose
 * distance sum took the one-lane serial chain (hough_peak.hip: the in-order
 * fp32 sum is rebuilt in parallel and verified; the serial chain is the
 * fallback when a verification fails; same bits either way).  Synchronous
 * (reads device memory).  The environment variable PCNN_HOUGH_SUM=serial
 * forces the serial chain for every maximum (A/B and test knob). */
int pcnn_hough_voting_diag(const void* workspace, int B, int H, int W, int C, int skip_pixels, float vote_thr,
                           int32_t* diag_host4, void* stream);

/* ---------------------------------------------------------------------------
 * RoI max pooling (RoiPool / RoiPoolGrad).
 * Replaces ROIPoolForwardLaucher / ROIPoolBackwardLaucher
 * (lib/roi_pooling_layer/roi_pooling_op_gpu.cu.cc:103-131, :232-254;
 *  called from roi_pooling_op.cc:250-254, :358-361).
 *  layout 0 = NHWC data (B,H,W,C), output (R,PH,PW,Cout)  [TF op]
 *  layout 1 = NCHW data (B,C,H,W), output (R,Cout,PH,PW)  [my_tools _RoIPooling]
 *  rois (R_cap, roi_stride) rows [b, cls, x1, y1, x2, y2, ...] (roi_stride >= 6), or
 *       with roi_stride == 5 rows [b, x1, y1, x2, y2] (pth API, class column absent)
 *  batch_base: subtracted from the rows' batch column to index `data` (an
 *       image-sharded rank holds images [batch_base, batch_base + B) of the
 *       global batch and the Hough rows carry the global index; 0 otherwise)
 *  num_rois_dev: optional device int; when non-NULL the row count is
 *       min(*num_rois_dev, R_cap) (rows beyond are not touched)
 *  argmax: flat index within the image, (h*W + w)*C + c (NHWC) or (c*H + h)*W + w (NCHW)
 * ------------------------------------------------------------------------- */
int pcnn_roi_pool_fwd(const float* data, int B, int H, int W, int C, int layout, const float* rois, int R_cap,
                      int roi_stride, int batch_base, const int32_t* num_rois_dev, float spatial_scale, int pooled_h, int pooled_w,
                      int pool_channel, float* top, int32_t* argmax, void* stream);

/* As pcnn_roi_pool_fwd but top += pooled (argmax is written as usual): the
 * second pool of vgg16_convs.py:178-184 produces pool5 + pool4 in place, so
 * the fc6 contraction reads one operand.  Same sum as tf.add(pool5, pool4). */
int pcnn_roi_pool_fwd_accumulate(const float* data, int B, int H, int W, int C, int layout, const float* rois,
                                 int R_cap, int roi_stride, int batch_base, const int32_t* num_rois_dev,
                                 float spatial_scale, int pooled_h, int pooled_w, int pool_channel, float* top,
                                 int32_t* argmax, void* stream);

/* Both pose-head RoI pools in one pass (vgg16_convs.py:177-184): pool5 on
 * data_a (e.g. conv5_3 at 1/16) and pool4 on data_b (conv4_3 at 1/8), NHWC,
 * all channels, C % 4 == 0, 16-B aligned. Writes top_sum = pool_a + pool_b
 * (one fp32 add per element, as pcnn_roi_pool_fwd then _accumulate) and both
 * argmax tensors (R_cap, pooled_h, pooled_w, C). */
int pcnn_roi_pool_fwd_pair(const float* data_a, int Ha, int Wa, float scale_a, const float* data_b, int Hb, int Wb,
                           float scale_b, int B, int C, const float* rois, int R_cap, int roi_stride,
                           int batch_base, const int32_t* num_rois_dev, int pooled_h, int pooled_w, float* top_sum,
                           int32_t* argmax_a, int32_t* argmax_b, void* stream);

/* pcnn_roi_pool_fwd_pair with the compact argmax of the fused pose step: per
 * output element the uint16 pixel index h*W + w of the max within its image
 * (the channel is the element's own; 0xFFFF = empty bin, so H*W < 0xFFFF for
 * both maps), i.e. the reference's flat index argmax = pixel*C + c
 * (roi_pooling_op_gpu.cu.cc:87-97) in half the bytes. argmax 8-B aligned.
 * Consumed by pcnn_roi_pool_bwd_px. */
int pcnn_roi_pool_fwd_pair_px(const float* data_a, int Ha, int Wa, float scale_a, const float* data_b, int Hb,
                              int Wb, float scale_b, int B, int C, const float* rois, int R_cap, int roi_stride,
                              int batch_base, const int32_t* num_rois_dev, int pooled_h, int pooled_w,
                              float* top_sum, uint16_t* argmax_a, uint16_t* argmax_b, void* stream);

size_t pcnn_roi_pool_bwd_workspace_size(int B, int R_cap);

int pcnn_roi_pool_bwd(const float* top_diff, const int32_t* argmax, int B, int H, int W, int C, int layout,
                      const float* rois, int R_cap, int roi_stride, int batch_base, const int32_t* num_rois_dev,
                      float spatial_scale, int pooled_h, int pooled_w, int pool_channel, float* bottom_diff,
                      void* workspace, size_t workspace_bytes, void* stream);

/* pcnn_roi_pool_bwd on the pixel-index argmax of pcnn_roi_pool_fwd_pair_px:
 * NHWC, all channels (pool_channel 0), C even, H*W < 0xFFFF; the same
 * entry-list gather and (RoI, ph, pw) summation order, so bit-equal to
 * pcnn_roi_pool_bwd on the flat argmax. */
int pcnn_roi_pool_bwd_px(const float* top_diff, const uint16_t* argmax_px, int B, int H, int W, int C,
                         const float* rois, int R_cap, int roi_stride, int batch_base, const int32_t* num_rois_dev,
                         float spatial_scale, int pooled_h, int pooled_w, float* bottom_diff, void* workspace,
                         size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * ADD / ADD-S pose loss (Averagedistance / AveragedistanceGrad).
 * Replaces AveragedistanceForwardLaucher / AveragedistanceBackwardLaucher
 * (lib/average_distance_loss/average_distance_loss_op_gpu.cu.cc:256-343, :357-377;
 *  called from average_distance_loss_op.cc:228-231, :362-363).
 *  pred/target/weight (R_cap, 4C), points (C,P,3), symmetry (C)
 *  loss (1) f32, bottom_diff (R_cap, 4C); rows counted from num_rois_dev when non-NULL.
 *  loss_norm_rows: when > 0, the normaliser R of (d - m)/(2 R P) and of the
 *       gradient (an image-sharded run passes the global row count so that the
 *       per-rank losses sum to the single-device loss); <= 0 uses the local R.
 * ------------------------------------------------------------------------- */
size_t pcnn_add_loss_workspace_size(int R_cap, int C, int P);

int pcnn_add_loss_fwd(const float* pred, const float* target, const float* weight, const float* points,
                      const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P, float margin,
                      int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss, float* bottom_diff,
                      void* workspace, size_t workspace_bytes, void* stream);

/* pcnn_add_loss_fwd split in two: pcnn_add_loss_prep classifies the rows
 * (first class with weight > 0, cu.cc:47-52; the symmetric-row list) from the
 * weights alone, so a caller may run it as soon as the Hough targets exist, on
 * another stream; pcnn_add_loss_fwd_prepared is then pcnn_add_loss_fwd without
 * that step, on the same workspace, weights and row count (ordered after the
 * prep by the caller). */
int pcnn_add_loss_prep(const float* weight, const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C,
                       int P, void* workspace, size_t workspace_bytes, void* stream);
/* pcnn_add_loss_prep with the model points (C, P, 3): when the environment
 * sets PCNN_ADD_SEARCH=pruned (P <= 4096) it also builds each symmetric
 * class's Morton order in the workspace, which the ADD-S nearest-point search
 * then prunes with (the same bits as the default full O(P^2) scan). */
/* Byte offset in the loss workspace of the pruned search's diagnostics
 * (what = 0: the Morton orders, C x P int32; 1: int32 [blocks scanned, blocks
 * held] of the last search), -1 when P is past the pruned search's limit. */
long pcnn_add_loss_ws_offset(int R_cap, int C, int P, int what);
int pcnn_add_loss_prep_points(const float* weight, const float* symmetry, const float* points, int R_cap,
                              const int32_t* num_rois_dev, int C, int P, void* workspace, size_t workspace_bytes,
                              void* stream);
int pcnn_add_loss_fwd_prepared(const float* pred, const float* target, const float* weight, const float* points,
                               const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P,
                               float margin, int loss_norm_rows, const int32_t* loss_norm_rows_dev, float* loss,
                               float* bottom_diff, void* workspace, size_t workspace_bytes, void* stream);

/* The fused pose step's loss tail (posecnn_amd/pipeline.py): the prepared
 * loss's per-point sums, then one pass that finishes each row's bottom_diff
 * and runs the pose head's backward on it (pcnn_pose_head_bwd with
 * d_pred = bottom_diff, scaled by d_pred_scale[0] -- the ADD gradient op,
 * cu.cc:346-354; tanh_out and poses_weight = weight as pcnn_pose_head_fwd
 * used them) into d_y8 (R, 4C): the same bits as pcnn_add_loss_fwd_prepared
 * + pcnn_pose_head_bwd.  The scalar loss is left to pcnn_add_loss_total on
 * the same workspace, which the caller may order on another stream (nothing
 * on the backward chain reads it).  4C <= 256. */
int pcnn_add_loss_fwd_head_bwd(const float* pred, const float* target, const float* weight, const float* points,
                               const float* symmetry, int R_cap, const int32_t* num_rois_dev, int C, int P,
                               float margin, int loss_norm_rows, const int32_t* loss_norm_rows_dev,
                               float* bottom_diff, void* workspace, size_t workspace_bytes, const float* tanh_out,
                               const float* d_pred_scale, float* d_y8, void* stream);
int pcnn_add_loss_total(int R_cap, const int32_t* num_rois_dev, int C, int P, const void* workspace,
                        size_t workspace_bytes, float* loss, void* stream);

/* out[i] = top_diff[0] * bottom_diff[i], n = rows * 4C */
int pcnn_add_loss_bwd(const float* top_diff, const float* bottom_diff, int n, const int32_t* num_rois_dev,
                      int row_len, float* out, void* stream);

/* Self-check of the ADD loss's per-launch division (average_distance.hip
 * div_rn): out[i] = x[i] / b correctly rounded, through the kernels' reciprocal
 * + two fma-correction form, in fp32 (dbl = 0) or in double rounded to fp32
 * (dbl = 1, the loss-sum form of cu.cc:181).  Test infrastructure only. */
int pcnn_div_rn_check(const float* x, float b, int n, int dbl, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Depth backprojection (Backproject / BackprojectGrad).
 * Replaces BackprojectForwardLaucher / BackprojectBackwardLaucher
 * (lib/backprojecting_layer/backprojecting_op_gpu.cu.cc:129-155, :220-242;
 *  called from backprojecting_op.cc:262-267, :388-390).
 *  data (B,H,W,Ch) label (B,H,W,NC) depth (B,H,W) meta (B,num_meta) label_3d (B,G,G,G,NC)
 *  -> top_data (B,G,G,G,Ch), top_label (B,G,G,G,NC), top_flag (B,G,G,G,Ch)
 * ------------------------------------------------------------------------- */
int pcnn_backproject_fwd(const float* data, const float* label, const float* depth, const float* meta, int num_meta,
                         const float* label_3d, int B, int H, int W, int Ch, int NC, int grid_size,
                         int kernel_size, float threshold, float* top_data, float* top_label, float* top_flag,
                         void* stream);

int pcnn_backproject_bwd(const float* top_diff, const float* depth, const float* meta, int num_meta, int B, int H,
                         int W, int Ch, int grid_size, float* bottom_diff, void* stream);

/* ---------------------------------------------------------------------------
 * Pose-head FC contraction (MFMA).  Replaces the TF matmuls of
 * Network.fc (lib/networks/network.py:393-423) as wired by vgg16_convs.py:186-197:
 *   C[M,N] = epilogue( op(A)[M,K] (+ op(A2)) * op(B)[K,N] )
 *  a_trans: 0 -> A stored (M,K) row-major (lda >= K); 1 -> A stored (K,M) (lda >= M)
 *  b_trans: 0 -> B stored (K,N) (ldb >= N);           1 -> B stored (N,K) (ldb >= K)
 *  A2 (optional): same layout as A, added elementwise (pool5 + pool4 fusion)
 *  M_dev / K_dev (optional device ints): effective M / K = min(*dev, M / K)
 *  epilogue: bias (N) added if non-NULL; act 0 none, 1 relu;
 *            mask (optional, ldm) -> C *= (mask > 0)  (relu backward)
 *  precision: 0 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32),
 *             1 = split-bf16 x3 MFMA (hi*hi + hi*lo + lo*hi: ~2^-16 per product),
 *             2 = exact three-way split-bf16 x6 MFMA (hi/mid/lo planes, six
 *                 products: within 2^-24 |a||b| per product, fp32
 *                 accumulation -- fp32-faithful; the pose step's default).
 *                 Operand range: finite |x| <= 3.3895314e38 (the largest bf16);
 *                 there results track fp32.  An inf / NaN operand, or a finite
 *                 one above that bound (its hi plane rounds to inf), makes the
 *                 output elements it reaches NaN (fp32 would give +-inf or a
 *                 finite value); every other element is unaffected
 *                 (tests/test_gpu_gemm_fc6.py::test_x6_edge_semantics).
 *  Deterministic (split-K partials are reduced in fixed order).
 *  workspace: >= pcnn_gemm_workspace_size() bytes, one per stream.
 * ------------------------------------------------------------------------- */
size_t pcnn_gemm_workspace_size(int M, int N, int K, int m_dynamic, int precision);

int pcnn_gemm(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B, int ldb,
              int b_trans, float* Cm, int ldc, const float* bias, int act, const float* mask, int ldm,
              const int32_t* M_dev, const int32_t* K_dev, int precision, void* workspace, size_t workspace_bytes,
              void* stream);

/* pcnn_gemm plus the pose head's dropout (drop6 / drop7, vgg16_convs.py:189,191;
 * Network.dropout = tf.nn.dropout, network.py:574-577; keep_prob 0.5 in
 * training, lib/fcn/train.py:421, 1.0 at test time, test.py:173):
 *  drop (optional, uint8 (M, ldd >= N), 0 / 1): forward, applied after bias / act
 *       as tf.nn.dropout computes it: C = (v / keep_prob) * drop
 *  mask (optional): backward of relu + dropout, with mask = the dropped
 *       forward activation: C = mask > 0 ? v / keep_prob : 0
 *       (TF: ReluGrad(features) of (grad * binary) / keep_prob)
 *  keep_prob in (0, 1]; 1 with drop == NULL is exactly pcnn_gemm. */
int pcnn_gemm_drop(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B,
                   int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act, const float* mask, int ldm,
                   const uint8_t* drop, int ldd, float keep_prob, const int32_t* M_dev, const int32_t* K_dev,
                   int precision, void* workspace, size_t workspace_bytes, void* stream);

/* The forward of pcnn_gemm_drop with the keep mask drawn in the epilogue: the
 * reduce pass draws, for every live element (m < effective M, n < N), the bit
 * pcnn_dropout_mask would write for a dense (M, N) mask with the same seed,
 * *step_dev and stream_id, applies C = (v / keep_prob) * bit, and stores the
 * bits into drop_out (uint8 (M, ldd)) for the backward (pcnn_gemm_drop with
 * mask).  Bit-identical to pcnn_dropout_mask (rows_dev = M_dev) followed by
 * pcnn_gemm_drop, without the mask launch.  N % 4 == 0, ldd % 4 == 0. */
int pcnn_gemm_drop_gen(int M, int N, int K, const float* A, const float* A2, int lda, int a_trans, const float* B,
                       int ldb, int b_trans, float* Cm, int ldc, const float* bias, int act, uint8_t* drop_out,
                       int ldd, float keep_prob, uint64_t seed, const int64_t* step_dev, int stream_id,
                       const int32_t* M_dev, const int32_t* K_dev, int precision, void* workspace,
                       size_t workspace_bytes, void* stream);

/* The x6 GEMM on pre-split operands (gemm_tp.hip), bit-identical to pcnn_gemm
 * precision 2 on the same fp32 values, with no split work in its K loop.
 * Tiled planes ("TP") of a rows x K operand: block (rb, ks) of 32 rows x 16 k
 * is 3 KiB at ((rb * ceil(K/16) + ks) * 3) KiB, planes hi / mid / lo (the exact
 * 3-way bf16 split), lane l of a plane holding row 32 rb + (l & 31),
 * k 16 ks + 8 (l >> 5) .. + 7 (the MFMA operand fragment).
 *  pcnn_tp_bytes: storage of one operand.
 *  pcnn_split_tp: dst <- TP of the fp32 view src[row * row_stride + k * k_stride]
 *    (rows, K capacities; effective counts from rows_dev / K_dev if non-NULL,
 *    zeros past them; row blocks past ceil(rows_eff / 32) and K steps past
 *    ceil(K_eff / 16) are never multiplied and not written).
 *  pcnn_gemm_tp: C[M,N] = epilogue(A · B) with A_tp = TP of op(A) (M x K) and
 *    B_tp = TP of op(B)^T (N x K), both stored at capacity K; epilogue, M_dev /
 *    K_dev, dropout and workspace as pcnn_gemm_drop at precision 2. */
size_t pcnn_tp_bytes(int rows, int K);
int pcnn_split_tp(const float* src, long row_stride, long k_stride, int rows, const int32_t* rows_dev, int K,
                  const int32_t* K_dev, void* dst, size_t dst_bytes, void* stream);
int pcnn_gemm_tp(int M, int N, int K, const void* A_tp, const void* B_tp, float* Cm, int ldc, const float* bias,
                 int act, const float* mask, int ldm, const uint8_t* drop, int ldd, float keep_prob,
                 const int32_t* M_dev, const int32_t* K_dev, void* workspace, size_t workspace_bytes, void* stream);

/* Dropout keep masks (the binary tensor of tf.nn.dropout: floor(keep_prob + U[0,1))):
 * mask[r, c] for r < min(*rows_dev, rows) (rows_dev may be NULL), c < cols, row
 * pitch ld >= cols bytes.  U comes from Philox4x32-10 (key = seed, counter =
 * (element quad index, *step_dev)) in TF's uint32 -> float construction
 * ((x & 0x7fffff) | 0x3f800000 as a float, minus 1).  The draw is keyed on the
 * device-side step counter, so a captured HIP graph draws new masks on every
 * replay.  TF's own stream assignment is not reproducible (parity unpinned:
 * the masks are i.i.d. Bernoulli(keep_prob) either way); several masks of one
 * step take distinct `stream_id`s.  cols % 4 == 0 and ld % 4 == 0. */
int pcnn_dropout_mask(uint8_t* mask, int rows, int cols, int ld, const int32_t* rows_dev, uint64_t seed,
                      const int64_t* step_dev, int stream_id, float keep_prob, void* stream);

/* Philox4x32-10 self-check (test infrastructure): out[4 i .. 4 i + 3] = philox(ctr[4 i .. 4 i + 3], key[2 i .. 2 i + 1]). */
int pcnn_philox_check(const uint32_t* ctr, const uint32_t* key, int n, uint32_t* out, void* stream);

/* ---------------------------------------------------------------------------
 * RGB-only pose estimation (the RANSAC half).
 * Replaces Synthesizer::estimatePose2D (lib/synthesize/synthesize.cpp:1571-1766;
 * synthesizer.pyx:74-82 estimate_poses_2d, called from lib/fcn/test.py:1364).
 *  label (H,W) int32, vertmap (H,W,3C) object coordinates scaled to [0,1] by the
 *  class extents (getMode3D, :1052-1071), extents (C,3), pinhole fx fy px py.
 *  Preemptive RANSAC: n_hyp (1..256; 256 = the reference's ransacIterations,
 *  :1601) hypotheses, each from 4 pixels of one object (> 400 pixels) through
 *  P3P; attempt a of hypothesis h draws on its own Philox stream (h, a) of
 *  `seed`, h keeps its first accepted attempt (at most max_iter attempts); 8
 *  rounds of inlier counting (< 10 px) over pixel subsets with the
 *  reference's skip law max(1, G), G geometric with p = 1000 r / N (drawn
 *  from Philox streams (j, class, round) of `seed`), keeping the better
 *  half.  Outputs (device): poses_out (3,4,C) [R | t] per class (the reference's
 *  layout; classes without a hypothesis 0); hyps_out (n_hyp,13) [objID or -1 |
 *  R | t]; hyp_px (n_hyp,4) sampled pixel indices; inl_out (n_hyp,8) inliers per
 *  round (-1: not queued); final_out (C,3) [h, inliers, hypotheses] (-1: none).
 *  Asynchronous on `stream`: object lists and subsets are built on the device. */
size_t pcnn_pose2d_workspace_size(int H, int W, int C, int n_hyp);
int pcnn_pose2d(const int32_t* label, const float* vertmap, const float* extents, int H, int W, int C, float fx,
                float fy, float px, float py, uint64_t seed, int n_hyp, int max_iter, float* poses_out,
                float* hyps_out, int32_t* hyp_px, int32_t* inl_out, int32_t* final_out, void* workspace,
                size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Depth-based pose estimation (the cfg.TEST.VERTEX_REG_3D
 * branch).  Replaces Synthesizer::estimatePose3D (lib/synthesize/synthesize.cpp:
 * 1769-1965; synthesizer.pyx:86-95 estimate_poses_3d, called from
 * lib/fcn/test.py:1385, its poses then refined by solveICP, test.py:1403-1416).
 *  label, vertmap, extents, fx fy px py as pcnn_pose2d; depth (H,W) uint16 raw
 *  depth, camera coordinates = pxToEye (:1372-1389) with depth_factor.
 *  Preemptive RANSAC over 3-D / 3-D correspondences: n_hyp (1..256) hypotheses,
 *  each from 3 pixels of one object with depth through the rigid (Kabsch)
 *  transform, 1 cm reconstruction and 400 px box-area checks (attempt a of
 *  hypothesis h on Philox stream (h, 'P3D', a)); 8 rounds of inlier counting
 *  (< 1 cm) over hole-skipping pixel subsets (the pcnn_pose2d skip law), the
 *  better half kept, then updateHyp3D's refit on at most 1000 inliers
 *  (filterInliers3D picks on streams (h, 'F3D', 1024 r + k)); the survivor with
 *  more than 10 inliers refined by a bounded Nelder-Mead (nm_evals evaluations,
 *  100 in the reference) of optEnergy3D over (Rodrigues vector, t).
 *  Outputs (device): poses_out (3,4,C); hyps_out (n_hyp,13); hyp_px (n_hyp,3);
 *  inl_out (n_hyp,8); final_out (C,3) as pcnn_pose2d; energy_out (C) the
 *  refined optEnergy3D (0: not refined); eye_out (H,W,3) camera coordinates,
 *  optional (NULL: not written).  Asynchronous on `stream`. */
size_t pcnn_pose3d_workspace_size(int H, int W, int C, int n_hyp);
int pcnn_pose3d(const int32_t* label, const uint16_t* depth, const float* vertmap, const float* extents, int H, int W,
                int C, float fx, float fy, float px, float py, float depth_factor, uint64_t seed, int n_hyp,
                int max_iter, int nm_evals, float* poses_out, float* hyps_out, int32_t* hyp_px, int32_t* inl_out,
                int32_t* final_out, float* energy_out, float* eye_out, void* workspace, size_t workspace_bytes,
                void* stream);

/* Column sums over the first min(*M_dev, M) rows: out[n] = sum_m X[m, n] (bias gradients). */
int pcnn_colsum(const float* X, int M, int N, int ldx, const int32_t* M_dev, float* out, void* stream);

/* Pose-head tail (vgg16_convs.py:193-197): T = tanh(Y8); Mw = T * poses_weight;
 * pred = Mw / sqrt(max(sum(Mw^2), 1e-12)) (tf.nn.l2_normalize, dim 1).  Rows (R_cap, D). */
int pcnn_pose_head_fwd(const float* y8, const float* poses_weight, int R_cap, const int32_t* num_rois_dev, int D,
                       float* tanh_out, float* pred, void* stream);

/* Backward of the tail: d_pred -> d_y8 (through l2_normalize, multiply, tanh).
 * d_pred_scale (optional device scalar): d_pred is taken as d_pred_scale[0] * d_pred,
 * i.e. the ADD-loss gradient op (AveragedistanceBackward, average_distance_loss_op_gpu.cu.cc:346-354:
 * top_diff[0] * bottom_diff) folded into this pass; NULL = d_pred as given. */
int pcnn_pose_head_bwd(const float* d_pred, const float* d_pred_scale, const float* tanh_out,
                       const float* poses_weight, const float* pred, int R_cap, const int32_t* num_rois_dev, int D,
                       float* d_y8, void* stream);

/* ---------------------------------------------------------------------------
 * Class-aware greedy box NMS + pose combination (inference consumer of the
 * Hough rows).
 * Replaces lib/utils/nms.py:3-32 (numpy, on the host after a D2H copy) and the
 * pose combination of lib/fcn/test.py:197-211.
 *  rois (R_cap, roi_stride >= 7) [b,cls,x1,y1,x2,y2,score], row count from
 *  num_rois_dev (may be NULL: R_cap rows), R_cap <= 1152 (MAX_ROI * 9).
 *  keep (R_cap) int32: kept row indices, score descending (ties: lower row
 *  first — numpy argsort()[::-1] leaves tie order unspecified); num_keep (1).
 *  Optional (NULL to skip): rois_out (R_cap,7) = rois[keep]; poses_out (R_cap,7)
 *  = poses_init[keep] with [:4] = poses_pred[keep, 4*cls : 4*cls+4] for cls >= 0
 *  (poses_pred rows of pred_dim floats). Overlap test and areas in float32 in
 *  nms.py's operation order; suppression needs ovr > thresh and equal class.
 * ------------------------------------------------------------------------- */
int pcnn_box_nms(const float* rois, int R_cap, int roi_stride, const int32_t* num_rois_dev, float thresh,
                 int32_t* keep, int32_t* num_keep, const float* poses_init, const float* poses_pred, int pred_dim,
                 float* rois_out, float* poses_out, void* stream);

/* ---------------------------------------------------------------------------
 * Label producers.
 * argmax_2d: label (B,H,W) int32 = argmax over the last axis of prob (B,H,W,C)
 *   (lib/networks/network.py:433-434 `tf.to_int32(tf.argmax(input, 3))`);
 *   first maximum, a NaN wins at its first occurrence (numpy / tf.argmax).
 * Hardlabel: replaces HardlabelForwardLaucher / HardlabelBackwardLaucher
 *   (lib/hard_label_layer/hard_label_op_gpu.cu.cc:17-29,32-52,56-90; op
 *   hard_label_op.cc:30-44). top (B,H,W,C) = one-hot of gt where gt != -1 and
 *   (gt > 0 or prob[gt] < threshold), else 0; threshold > 0 (the op's attr
 *   check). gt outside [-1, C) (out-of-row store in the reference) -> zero row.
 *   Backward: zero gradients for prob (B,H,W,C) and gt (B,H,W) (either NULL).
 * ------------------------------------------------------------------------- */
int pcnn_argmax_2d(const float* prob, int B, int H, int W, int C, int32_t* label, void* stream);
int pcnn_hard_label_fwd(const float* prob, const int32_t* gt, int B, int H, int W, int C, float threshold,
                        float* top, void* stream);
int pcnn_hard_label_bwd(float* grad_prob, float* grad_gt, int B, int H, int W, int C, void* stream);

/* vertex_pred (vgg16_convs.py:152-163: 1x1 conv K -> 3C + bias_add,
 * network.py:168-185) evaluated only at each pixel's label class (SURVEY
 * §8(f) row 3): feat (B,H,W,K) NHWC, K % 4 == 0, weights (K,3C) as the
 * reference's [1,1,K,3C] kernel, bias (3C), label (B,H,W) -> vertex3 (B,H,W,3)
 * = (sum_k feat[k] * w[k][3l+j] in k order) + bias[3l+j]; zeros for labels
 * outside [0, C). K * 3C * 4 B <= 64 KiB. */
int pcnn_vertex_pred_compact(const float* feat, const float* weights, const float* bias, const int32_t* label, int B,
                             int H, int W, int K, int C, float* vertex3, void* stream);

/* ---------------------------------------------------------------------------
 * Test-time pose refinement: the numerical core of
 * Synthesizer::solveICP (lib/synthesize/synthesize.cpp:2052-2395, reached from
 * lib/fcn/test.py:1316-1351 via synthesizer.icp_python, synthesizer.pyx:60-75).
 * Maps are row-major (H,W,ch) f32; the rendered maps (the reference's OpenGL
 * pass, synthesize.cpp:2106-2137) are inputs: pred_vertices / pred_normals
 * (H,W,4) per problem (renderer_vn_ textures), vertmap (H,W,3) canonical model
 * coordinates with the class id in the integer part of x (renderer_ texture).
 * Poses are (qw,qx,qy,qz,tx,ty,tz); input quaternions are normalised as
 * Sophus' SE3(quaternion, translation) constructor does.
 *
 * pcnn_icp_live_vertices: live (L,H,W,3) = df::backproject of the masked depth
 *   (synthesize.cpp:2140-2160; backprojection.cu:10-27, Poly3 camera at zero
 *   distortion): d = depth / factor where label == obj_ids[l], else 0;
 *   vertex = ((x-px)/fx*d, (y-py)/fy*d, d). depth (H,W) uint16, H*W % 4 == 0.
 * pcnn_icp: df::icp (lib/kinect_fusion/src/optimization/icp.cpp:20-106 +
 *   icp.cu:22-245) for N problems: `iterations` Gauss-Newton steps of the
 *   projective point-to-plane residual (border 2 px, ray/normal test 0.1,
 *   |error| <= max_error, weight 1/live depth), each solving JTJ x = JTr
 *   (Eigen LDLT) and left-multiplying SE3::exp(x) into the accumulated update.
 *   live (num_live,H,W,3) with live_index (N) selecting problem n's map (NULL:
 *   n; an index outside [0, num_live) contributes no pixel);
 *   update (N,7); pose_in / pose_out (N,7) optional: pose_out = update * pose_in
 *   (refinePose, synthesize.cpp:2023-2025); systems (N,iterations,28) optional:
 *   per iteration the 21 upper-triangle JTJ entries, 6 JTr and the pixel count.
 * pcnn_icp_center: the translation re-centring of solveICP
 *   (synthesize.cpp:2163-2219) for L objects: out (L,4) = mean(live - model) over
 *   the object's pixels with depth > 0, finite vertmap and |n.(live - pred)| <
 *   max_error, and the count; pose_out = pose_in with t = (rx Tz, ry Tz, Tz),
 *   rx = tx / tz of pose_in, when the count is > 0.
 * pcnn_pose_energy: optEnergy (synthesize.cpp:2474-2526) of K poses: mean
 *   |T p - v| over the object's pixels with finite T p and both depths inside
 *   (znear, zfar); energy (K).
 * ------------------------------------------------------------------------- */
int pcnn_icp_live_vertices(const uint16_t* depth, const int32_t* label, int H, int W, const int32_t* obj_ids, int L,
                           float factor, float fx, float fy, float px, float py, float* live, void* stream);
size_t pcnn_icp_workspace_size(int N, int H, int W);
int pcnn_icp(const float* live, int num_live, const int32_t* live_index, const float* pred_vertices,
             const float* pred_normals, int N, int H, int W, float fx, float fy, float px, float py, float znear, float zfar, float max_error,
             int iterations, const float* pose_in, float* update, float* pose_out, float* systems, void* workspace,
             size_t workspace_bytes, void* stream);
size_t pcnn_icp_reduce_workspace_size(int L, int H, int W);
int pcnn_icp_center(const float* live, const int32_t* label, const int32_t* obj_ids, int L, const float* vertmap,
                    const float* pred_vertices, const float* pred_normals, int H, int W, float max_error,
                    const float* pose_in, float* out, float* pose_out, void* workspace, size_t workspace_bytes,
                    void* stream);
/* Nelder-Mead on optEnergy on the device (round 5): solveICP's refinePose
 * search (synthesize.cpp:2221-2250 -> poseWithOpt :2529-2573, NLopt
 * LN_NELDERMEAD over 7 parameters, optEnergy :2476-2526).
 *  pcnn_energy_records: for problem i (N), the pixels with label ==
 *  prob_obj[i] whose live vertex (live (n_live,H,W,3)[prob_live[i]]) has z in
 *  (znear, zfar), in raster order, as records (rendered vertex
 *  pred_vertices (N,H,W,4)[i] xyz, live xyz) -> records (N, H*W, 6), counts (N).
 *  pcnn_energy_rec: optEnergy of K poses (K,7), pose k over problem
 *  pose_prob[k]'s records (stride = records per problem, H*W).
 *  pcnn_nelder_mead_energy: N bounded Nelder-Mead searches (x0, lb, ub (N,7)
 *  float64, at most max_eval evaluations; the operation order of
 *  posecnn_amd/synthesize/icp.py nelder_mead_steps), one workgroup each, the
 *  energy of every trial point as pcnn_energy_rec computes it (the same bits)
 *  -> x_out (N,7), f_out (N) float64, nev_out (N). Asynchronous. */
size_t pcnn_energy_records_workspace_size(int N, int H, int W);
int pcnn_energy_records(const float* live, int n_live, const int32_t* label, const float* pred_vertices, int H, int W,
                        float znear, float zfar, int N, const int32_t* prob_obj, const int32_t* prob_live,
                        float* records, int32_t* counts, void* workspace, size_t workspace_bytes, void* stream);
int pcnn_energy_rec(const float* records, const int32_t* counts, int stride, const float* poses,
                    const int32_t* pose_prob, int K, float znear, float zfar, float* energy, void* stream);
int pcnn_nelder_mead_energy(const float* records, const int32_t* counts, int stride, int N, const double* x0,
                            const double* lb, const double* ub, int max_eval, float znear, float zfar, double* x_out,
                            double* f_out, int32_t* nev_out, void* stream);

/* pcnn_nelder_mead_energy with 8 cooperating workgroups per evaluated point
 * (the evaluation's records spread over 8 CUs, one arrive-and-wait per round
 * through the workspace), launched cooperatively; the same bits.  N <= 32:
 * speculative rounds (an iteration's reflection, expansion and both
 * contractions evaluated together by 4 x 8 workgroups, the search counting
 * only those it uses); N <= 128: one point per round.  The workspace holds
 * the wave sums, one arrival counter and one failure flag per problem
 * (zeroed by the call).  nev_out = -1 marks a problem one of whose
 * cross-workgroup waits gave up: every workgroup of it stops at its next
 * barrier and its x / f are invalid.  max_eval >= 8 (the initial simplex;
 * NLopt's maxeval, which poseWithOpt / refineWithOpt set, counts it too).
 * The _path form pins the kernel (force_path 1 speculative, 2 cooperative,
 * 3 one workgroup; 0 the first that launches) and reports the one that ran
 * in *path_out (host int, may be NULL); PCNN_EHIP if a forced one cannot
 * launch. */
size_t pcnn_nelder_mead_energy_workspace_size(int N);
int pcnn_nelder_mead_energy_coop(const float* records, const int32_t* counts, int stride, int N, const double* x0,
                                 const double* lb, const double* ub, int max_eval, float znear, float zfar,
                                 double* x_out, double* f_out, int32_t* nev_out, void* workspace,
                                 size_t workspace_bytes, void* stream);
int pcnn_nelder_mead_energy_coop_path(const float* records, const int32_t* counts, int stride, int N,
                                      const double* x0, const double* lb, const double* ub, int max_eval,
                                      float znear, float zfar, double* x_out, double* f_out, int32_t* nev_out,
                                      void* workspace, size_t workspace_bytes, int force_path, int32_t* path_out,
                                      void* stream);

/* pcnn_icp_score: the SegICP hypothesis score of solveICP (synthesize.cpp:2288-2330):
 *   over the object's pixels with depth > 0 and a finite vertmap, each model
 *   point (vertmap, class offset dropped) moved by hypothesis j takes its
 *   nearest live point within `radius` (squared distance < radius^2; ties ->
 *   lowest raster index); score (J) = distinct live points taken / model points;
 *   choose (1) = first best hypothesis (0 when the object has no such pixel).
 *   J <= 64. */
size_t pcnn_icp_score_workspace_size(int J, int H, int W);
int pcnn_icp_score(const float* live, const int32_t* label, int obj, const float* vertmap, int H, int W,
                   const float* hyps, int J, float radius, float* score, int32_t* choose, void* workspace,
                   size_t workspace_bytes, void* stream);
int pcnn_pose_energy(const float* live, const int32_t* label, int obj, const float* pred_vertices, int H, int W,
                     float znear, float zfar, const float* poses, int K, float* energy, void* workspace,
                     size_t workspace_bytes, void* stream);

/* Batched optEnergy: pose k (of K) is scored for object pose_obj[k] against live
 * map pose_live[k] (of n_live, (H,W,3) each) and rendered vertices pose_pv[k]
 * (of n_pv, (H,W,4) each) -- one launch for the Nelder-Mead simplices of every
 * RoI of solveICP (synthesize.cpp:2529-2573), which the reference evaluates one
 * pose at a time.  workspace: pcnn_icp_reduce_workspace_size(K, H, W). */
int pcnn_pose_energy_batch(const float* live, int n_live, const int32_t* label, const float* pred_vertices, int n_pv,
                           int H, int W, float znear, float zfar, const float* poses, int K, const int32_t* pose_obj,
                           const int32_t* pose_live, const int32_t* pose_pv, float* energy, void* workspace,
                           size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POSECNN_HIP_H */
