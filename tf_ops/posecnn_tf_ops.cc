// TensorFlow custom-op binding of the MI355X hot path (TF-ROCm only): the
// reference's op names, attributes, inputs and outputs, with every GPU kernel
// class's Compute calling the C-ABI of libposecnn_hip.so (include/posecnn_hip.h).
//
// Registrations mirror (interface, not implementation):
//   Houghvotinggpu / HoughvotinggpuGrad  lib/hough_voting_gpu_layer/hough_voting_gpu_op.cc:37-60
//   RoiPool / RoiPoolGrad                lib/roi_pooling_layer/roi_pooling_op.cc:29-50
//   Averagedistance / AveragedistanceGrad lib/average_distance_loss/average_distance_loss_op.cc:38-54
//   Backproject / BackprojectGrad        lib/backprojecting_layer/backprojecting_op.cc:30-53
// Only the GPU kernels are registered (the reference's GPU kernels are float
// only too: hough_voting_gpu_op.cc:437, roi_pooling_op.cc:355, ...).  Shape
// functions stay in the reference's Python *_op_grad.py (ops.RegisterShape),
// as there.  Build: tf_ops/build_tf_ops.py (skipped when TensorFlow is absent).
//
// Differences from the reference kernels that a caller can observe: none in
// the outputs (they are the parity-tested C-ABI results); errors come back as
// OP_REQUIRES failures instead of exit(-1); no host sync except the
// Hough op's single row-count read, which the reference also does
// (hough_voting_gpu_op.cc:380).
#include "tensorflow/core/framework/op.h"
#include "tensorflow/core/framework/op_kernel.h"
#include "tensorflow/core/framework/tensor_shape.h"
#include <hip/hip_runtime_api.h>

#include "posecnn_hip.h"

using namespace tensorflow;
using GPUDevice = Eigen::GpuDevice;

// ---------------------------------------------------------------------------
REGISTER_OP("Houghvotinggpu")
    .Attr("T: {float, double}")
    .Attr("is_train: int")
    .Attr("threshold_vote: float")
    .Attr("threshold_percentage: float")
    .Attr("skip_pixels: int")
    .Input("bottom_label: int32")
    .Input("bottom_vertex: T")
    .Input("bottom_extents: T")
    .Input("bottom_meta_data: T")
    .Input("bottom_gt: T")
    .Output("top_box: T")
    .Output("top_pose: T")
    .Output("top_target: T")
    .Output("top_weight: T")
    .Output("top_domain: int32");

REGISTER_OP("HoughvotinggpuGrad")
    .Attr("T: {float, double}")
    .Input("bottom_label: int32")
    .Input("bottom_vertex: T")
    .Input("grad: T")
    .Output("output_label: T")
    .Output("output_vertex: T");

REGISTER_OP("RoiPool")
    .Attr("T: {float, double}")
    .Attr("pooled_height: int")
    .Attr("pooled_width: int")
    .Attr("spatial_scale: float")
    .Attr("pool_channel: int")
    .Input("bottom_data: T")
    .Input("bottom_rois: T")
    .Output("top_data: T")
    .Output("argmax: int32");

REGISTER_OP("RoiPoolGrad")
    .Attr("T: {float, double}")
    .Attr("pooled_height: int")
    .Attr("pooled_width: int")
    .Attr("spatial_scale: float")
    .Attr("pool_channel: int")
    .Input("bottom_data: T")
    .Input("bottom_rois: T")
    .Input("argmax: int32")
    .Input("grad: T")
    .Output("output: T");

REGISTER_OP("Averagedistance")
    .Attr("T: {float, double}")
    .Attr("margin: float")
    .Input("bottom_prediction: T")
    .Input("bottom_target: T")
    .Input("bottom_weight: T")
    .Input("bottom_point: T")
    .Input("bottom_symmetry: T")
    .Output("loss: T")
    .Output("bottom_diff: T");

REGISTER_OP("AveragedistanceGrad")
    .Attr("T: {float, double}")
    .Attr("margin: float")
    .Input("bottom_diff: T")
    .Input("grad: T")
    .Output("output: T");

REGISTER_OP("Backproject")
    .Attr("T: {float, double}")
    .Attr("grid_size: int")
    .Attr("kernel_size: int")
    .Attr("threshold: float")
    .Input("bottom_data: T")
    .Input("bottom_label: T")
    .Input("bottom_depth: T")
    .Input("bottom_meta_data: T")
    .Input("bottom_label_3d: T")
    .Output("top_data: T")
    .Output("top_label: T")
    .Output("top_flag: T");

REGISTER_OP("BackprojectGrad")
    .Attr("T: {float, double}")
    .Attr("grid_size: int")
    .Attr("kernel_size: int")
    .Attr("threshold: float")
    .Input("bottom_data: T")
    .Input("bottom_depth: T")
    .Input("bottom_meta_data: T")
    .Input("grad: T")
    .Output("output: T");

// ---------------------------------------------------------------------------
namespace {

void* stream_of(OpKernelContext* ctx) { return (void*)ctx->eigen_device<GPUDevice>().stream(); }

#define PCNN_TF_CHECK(ctx, call)                                                                  \
  do {                                                                                            \
    const int rc_ = (call);                                                                       \
    OP_REQUIRES(ctx, rc_ == PCNN_OK,                                                              \
                rc_ == PCNN_EINVAL ? errors::InvalidArgument(pcnn_strerror(rc_))                  \
                                   : errors::Internal(pcnn_strerror(rc_)));                       \
  } while (0)

Status temp_bytes(OpKernelContext* ctx, size_t n, Tensor* t) {
  return ctx->allocate_temp(DT_UINT8, TensorShape({static_cast<int64_t>(n > 0 ? n : 1)}), t);
}

// Houghvotinggpu: capacity-sized temps (MAX_ROI * 9 rows, hough_voting_gpu_op.cc:92-122),
// one call for the whole batch, one D2H read of the row count, exact-size outputs.
class HoughvotinggpuOp : public OpKernel {
 public:
  explicit HoughvotinggpuOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("is_train", &is_train_));
    OP_REQUIRES_OK(c, c->GetAttr("threshold_vote", &threshold_vote_));
    OP_REQUIRES_OK(c, c->GetAttr("threshold_percentage", &threshold_percentage_));
    OP_REQUIRES_OK(c, c->GetAttr("skip_pixels", &skip_pixels_));
  }

  void Compute(OpKernelContext* ctx) override {
    const Tensor& label = ctx->input(0);
    const Tensor& vertex = ctx->input(1);
    const Tensor& extents = ctx->input(2);
    const Tensor& meta = ctx->input(3);
    const Tensor& gt = ctx->input(4);
    OP_REQUIRES(ctx, label.dims() == 3, errors::InvalidArgument("label must be 3-dimensional"));
    OP_REQUIRES(ctx, vertex.dims() == 4, errors::InvalidArgument("vertex must be 4-dimensional"));
    const int B = label.dim_size(0), H = label.dim_size(1), W = label.dim_size(2);
    const int C = vertex.dim_size(3) / 3;
    const int cap = PCNN_MAX_ROI * 9;
    const int num_meta = meta.dims() == 4 ? meta.dim_size(3) : (int)(meta.NumElements() / (B > 0 ? B : 1));
    Tensor box, pose, target, weight, domain, count, ws;
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_FLOAT, TensorShape({cap, 7}), &box));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_FLOAT, TensorShape({cap, 7}), &pose));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_FLOAT, TensorShape({cap, 4 * C}), &target));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_FLOAT, TensorShape({cap, 4 * C}), &weight));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_INT32, TensorShape({cap}), &domain));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_INT32, TensorShape({2}), &count));
    const size_t wsb = pcnn_hough_voting_workspace_size(B, H, W, C, skip_pixels_, threshold_vote_);
    OP_REQUIRES_OK(ctx, temp_bytes(ctx, wsb, &ws));
    void* st = stream_of(ctx);
    // inlierThreshold 0.9 and labelThreshold 500 are the reference's hard-coded values (:356-357)
    PCNN_TF_CHECK(ctx, pcnn_hough_voting(label.flat<int32>().data(), vertex.flat<float>().data(),
                                         extents.flat<float>().data(), meta.flat<float>().data(), num_meta,
                                         gt.NumElements() ? gt.flat<float>().data() : nullptr, gt.dim_size(0), B, H, W,
                                         C, 0, B, is_train_, 0.9f, 500, threshold_vote_, threshold_percentage_,
                                         skip_pixels_, box.flat<float>().data(), pose.flat<float>().data(),
                                         target.flat<float>().data(), weight.flat<float>().data(),
                                         domain.flat<int32>().data(), count.flat<int32>().data(), cap, nullptr,
                                         ws.flat<uint8>().data(), wsb, st));
    int32 n[2] = {0, 0};
    OP_REQUIRES(ctx,
                hipMemcpyAsync(n, count.flat<int32>().data(), sizeof(n), hipMemcpyDeviceToHost,
                               (hipStream_t)st) == hipSuccess &&
                    hipStreamSynchronize((hipStream_t)st) == hipSuccess,
                errors::Internal("row count read failed"));
    const int rows = n[1];  // incl. the one zero row when nothing was detected (:382-383)
    const Tensor* temps[5] = {&box, &pose, &target, &weight, &domain};
    const int widths[5] = {7, 7, 4 * C, 4 * C, 0};
    for (int o = 0; o < 5; o++) {
      Tensor* out = nullptr;
      const TensorShape shp = widths[o] ? TensorShape({rows, widths[o]}) : TensorShape({rows});
      OP_REQUIRES_OK(ctx, ctx->allocate_output(o, shp, &out));
      const size_t bytes = (size_t)rows * (widths[o] ? widths[o] : 1) * 4;
      if (bytes)
        OP_REQUIRES(ctx,
                    hipMemcpyAsync(out->data(), temps[o]->data(), bytes, hipMemcpyDeviceToDevice, (hipStream_t)st) ==
                        hipSuccess,
                    errors::Internal("output copy failed"));
    }
  }

 private:
  int is_train_, skip_pixels_;
  float threshold_vote_, threshold_percentage_;
};

// HoughvotinggpuGrad: zeros (set_gradients, hough_voting_gpu_op.cu.cc:608-612)
class HoughvotinggpuGradOp : public OpKernel {
 public:
  explicit HoughvotinggpuGradOp(OpKernelConstruction* c) : OpKernel(c) {}
  void Compute(OpKernelContext* ctx) override {
    const Tensor& label = ctx->input(0);
    const Tensor& vertex = ctx->input(1);
    OP_REQUIRES(ctx, label.dims() == 3, errors::InvalidArgument("label must be 3-dimensional"));
    OP_REQUIRES(ctx, vertex.dims() == 4, errors::InvalidArgument("vertex must be 4-dimensional"));
    Tensor *gl = nullptr, *gv = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, label.shape(), &gl));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, vertex.shape(), &gv));
    PCNN_TF_CHECK(ctx, pcnn_hough_voting_grad(gl->flat<float>().data(), gv->flat<float>().data(), label.dim_size(0),
                                              label.dim_size(1), label.dim_size(2), vertex.dim_size(3) / 3,
                                              stream_of(ctx)));
  }
};

class RoiPoolOp : public OpKernel {
 public:
  explicit RoiPoolOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("pooled_height", &ph_));
    OP_REQUIRES_OK(c, c->GetAttr("pooled_width", &pw_));
    OP_REQUIRES_OK(c, c->GetAttr("spatial_scale", &scale_));
    OP_REQUIRES_OK(c, c->GetAttr("pool_channel", &pool_channel_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& data = ctx->input(0);
    const Tensor& rois = ctx->input(1);
    OP_REQUIRES(ctx, data.dims() == 4, errors::InvalidArgument("data must be 4-dimensional"));
    OP_REQUIRES(ctx, rois.dims() == 2, errors::InvalidArgument("rois must be 2-dimensional"));
    const int R = rois.dim_size(0), B = data.dim_size(0), H = data.dim_size(1), W = data.dim_size(2),
              C = data.dim_size(3);
    const TensorShape shp({R, ph_, pw_, pool_channel_ == 1 ? 1 : C});  // roi_pooling_op.cc:331-340
    Tensor *top = nullptr, *arg = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, shp, &top));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, shp, &arg));
    PCNN_TF_CHECK(ctx, pcnn_roi_pool_fwd(data.flat<float>().data(), B, H, W, C, 0, rois.flat<float>().data(), R,
                                         rois.dim_size(1), 0, nullptr, scale_, ph_, pw_, pool_channel_,
                                         top->flat<float>().data(), arg->flat<int32>().data(), stream_of(ctx)));
  }

 private:
  int ph_, pw_, pool_channel_;
  float scale_;
};

class RoiPoolGradOp : public OpKernel {
 public:
  explicit RoiPoolGradOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("pooled_height", &ph_));
    OP_REQUIRES_OK(c, c->GetAttr("pooled_width", &pw_));
    OP_REQUIRES_OK(c, c->GetAttr("spatial_scale", &scale_));
    OP_REQUIRES_OK(c, c->GetAttr("pool_channel", &pool_channel_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& data = ctx->input(0);
    const Tensor& rois = ctx->input(1);
    const Tensor& argmax = ctx->input(2);
    const Tensor& grad = ctx->input(3);
    OP_REQUIRES(ctx, data.dims() == 4, errors::InvalidArgument("data must be 4-dimensional"));
    OP_REQUIRES(ctx, rois.dims() == 2, errors::InvalidArgument("rois must be 2-dimensional"));
    OP_REQUIRES(ctx, argmax.dims() == 4, errors::InvalidArgument("argmax_data must be 4-dimensional"));
    OP_REQUIRES(ctx, grad.dims() == 4, errors::InvalidArgument("out_backprop must be 4-dimensional"));
    const int R = rois.dim_size(0), B = data.dim_size(0), H = data.dim_size(1), W = data.dim_size(2),
              C = data.dim_size(3);
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, data.shape(), &out));
    Tensor ws;
    const size_t wsb = pcnn_roi_pool_bwd_workspace_size(B, R);
    OP_REQUIRES_OK(ctx, temp_bytes(ctx, wsb, &ws));
    PCNN_TF_CHECK(ctx, pcnn_roi_pool_bwd(grad.flat<float>().data(), argmax.flat<int32>().data(), B, H, W, C, 0,
                                         rois.flat<float>().data(), R, rois.dim_size(1), 0, nullptr, scale_, ph_, pw_,
                                         pool_channel_, out->flat<float>().data(), ws.flat<uint8>().data(), wsb,
                                         stream_of(ctx)));
  }

 private:
  int ph_, pw_, pool_channel_;
  float scale_;
};

class AveragedistanceOp : public OpKernel {
 public:
  explicit AveragedistanceOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("margin", &margin_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& pred = ctx->input(0);
    const Tensor& target = ctx->input(1);
    const Tensor& weight = ctx->input(2);
    const Tensor& point = ctx->input(3);
    const Tensor& symmetry = ctx->input(4);
    OP_REQUIRES(ctx, pred.dims() == 2, errors::InvalidArgument("prediction must be 2-dimensional"));
    OP_REQUIRES(ctx, target.dims() == 2, errors::InvalidArgument("target must be 2-dimensional"));
    OP_REQUIRES(ctx, weight.dims() == 2, errors::InvalidArgument("weight must be 2-dimensional"));
    OP_REQUIRES(ctx, point.dims() == 3, errors::InvalidArgument("point must be 3-dimensional"));
    OP_REQUIRES(ctx, symmetry.dims() == 1, errors::InvalidArgument("symmetry must be 1-dimensional"));
    const int R = pred.dim_size(0), C = point.dim_size(0), P = point.dim_size(1);
    Tensor *loss = nullptr, *diff = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({1}), &loss));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, pred.shape(), &diff));
    Tensor ws;
    const size_t wsb = pcnn_add_loss_workspace_size(R, C, P);
    OP_REQUIRES_OK(ctx, temp_bytes(ctx, wsb, &ws));
    // loss normaliser = this op's row count (loss_norm_rows 0, cu.cc:181)
    PCNN_TF_CHECK(ctx, pcnn_add_loss_fwd(pred.flat<float>().data(), target.flat<float>().data(),
                                         weight.flat<float>().data(), point.flat<float>().data(),
                                         symmetry.flat<float>().data(), R, nullptr, C, P, margin_, 0, nullptr,
                                         loss->flat<float>().data(), diff->flat<float>().data(),
                                         ws.flat<uint8>().data(), wsb, stream_of(ctx)));
  }

 private:
  float margin_;
};

class AveragedistanceGradOp : public OpKernel {
 public:
  explicit AveragedistanceGradOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("margin", &margin_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& diff = ctx->input(0);
    const Tensor& grad = ctx->input(1);
    OP_REQUIRES(ctx, diff.dims() == 2, errors::InvalidArgument("bottom diff must be 2-dimensional"));
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, diff.shape(), &out));
    // output = grad[0] * bottom_diff (average_distance_loss_op_gpu.cu.cc:346-354)
    PCNN_TF_CHECK(ctx, pcnn_add_loss_bwd(grad.flat<float>().data(), diff.flat<float>().data(),
                                         (int)diff.NumElements(), nullptr, diff.dim_size(1),
                                         out->flat<float>().data(), stream_of(ctx)));
  }

 private:
  float margin_;
};

class BackprojectOp : public OpKernel {
 public:
  explicit BackprojectOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("grid_size", &grid_));
    OP_REQUIRES_OK(c, c->GetAttr("kernel_size", &kernel_));
    OP_REQUIRES_OK(c, c->GetAttr("threshold", &threshold_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& data = ctx->input(0);
    const Tensor& label = ctx->input(1);
    const Tensor& depth = ctx->input(2);
    const Tensor& meta = ctx->input(3);
    const Tensor& label3d = ctx->input(4);
    OP_REQUIRES(ctx, data.dims() == 4, errors::InvalidArgument("data must be 4-dimensional"));
    OP_REQUIRES(ctx, label.dims() == 4, errors::InvalidArgument("label must be 4-dimensional"));
    OP_REQUIRES(ctx, depth.dims() == 4, errors::InvalidArgument("depth must be 4-dimensional"));
    OP_REQUIRES(ctx, meta.dims() == 4, errors::InvalidArgument("meta data must be 4-dimensional"));
    OP_REQUIRES(ctx, label3d.dims() == 5, errors::InvalidArgument("label 3D must be 5-dimensional"));
    const int B = data.dim_size(0), H = data.dim_size(1), W = data.dim_size(2), Ch = data.dim_size(3),
              NC = label.dim_size(3);
    Tensor *top = nullptr, *tlabel = nullptr, *tflag = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({B, grid_, grid_, grid_, Ch}), &top));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, TensorShape({B, grid_, grid_, grid_, NC}), &tlabel));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(2, TensorShape({B, grid_, grid_, grid_, Ch}), &tflag));
    PCNN_TF_CHECK(ctx, pcnn_backproject_fwd(data.flat<float>().data(), label.flat<float>().data(),
                                            depth.flat<float>().data(), meta.flat<float>().data(), meta.dim_size(3),
                                            label3d.flat<float>().data(), B, H, W, Ch, NC, grid_, kernel_,
                                            threshold_, top->flat<float>().data(), tlabel->flat<float>().data(),
                                            tflag->flat<float>().data(), stream_of(ctx)));
  }

 private:
  int grid_, kernel_;
  float threshold_;
};

class BackprojectGradOp : public OpKernel {
 public:
  explicit BackprojectGradOp(OpKernelConstruction* c) : OpKernel(c) {
    OP_REQUIRES_OK(c, c->GetAttr("grid_size", &grid_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& data = ctx->input(0);
    const Tensor& depth = ctx->input(1);
    const Tensor& meta = ctx->input(2);
    const Tensor& grad = ctx->input(3);
    OP_REQUIRES(ctx, data.dims() == 4, errors::InvalidArgument("data must be 4-dimensional"));
    OP_REQUIRES(ctx, depth.dims() == 4, errors::InvalidArgument("depth must be 4-dimensional"));
    OP_REQUIRES(ctx, meta.dims() == 4, errors::InvalidArgument("meta data must be 4-dimensional"));
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, data.shape(), &out));
    PCNN_TF_CHECK(ctx, pcnn_backproject_bwd(grad.flat<float>().data(), depth.flat<float>().data(),
                                            meta.flat<float>().data(), meta.dim_size(3), data.dim_size(0),
                                            data.dim_size(1), data.dim_size(2), data.dim_size(3), grid_,
                                            out->flat<float>().data(), stream_of(ctx)));
  }

 private:
  int grid_;
};

}  // namespace

REGISTER_KERNEL_BUILDER(Name("Houghvotinggpu").Device(DEVICE_GPU).TypeConstraint<float>("T"), HoughvotinggpuOp);
REGISTER_KERNEL_BUILDER(Name("HoughvotinggpuGrad").Device(DEVICE_GPU).TypeConstraint<float>("T"), HoughvotinggpuGradOp);
REGISTER_KERNEL_BUILDER(Name("RoiPool").Device(DEVICE_GPU).TypeConstraint<float>("T"), RoiPoolOp);
REGISTER_KERNEL_BUILDER(Name("RoiPoolGrad").Device(DEVICE_GPU).TypeConstraint<float>("T"), RoiPoolGradOp);
REGISTER_KERNEL_BUILDER(Name("Averagedistance").Device(DEVICE_GPU).TypeConstraint<float>("T"), AveragedistanceOp);
REGISTER_KERNEL_BUILDER(Name("AveragedistanceGrad").Device(DEVICE_GPU).TypeConstraint<float>("T"),
                        AveragedistanceGradOp);
REGISTER_KERNEL_BUILDER(Name("Backproject").Device(DEVICE_GPU).TypeConstraint<float>("T"), BackprojectOp);
REGISTER_KERNEL_BUILDER(Name("BackprojectGrad").Device(DEVICE_GPU).TypeConstraint<float>("T"), BackprojectGradOp);
