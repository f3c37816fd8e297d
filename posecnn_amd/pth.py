"""The PyTorch module API the reference's my_tools scripts call
(my_tools/convert_to_pth.py:104-178, my_tools/loss_pth.py:51-64), backed by
the HIP ops of this package.  The reference imports these from a `lib/model`
package that it does not ship; the signatures here follow
its call sites:

    HoughVoting(num_classes, threshold_vote, threshold_percentage,
                label_threshold=500, inlier_threshold=0.9, skip_pixels=1,
                is_train=False)(label_2d, vertex_pred_NHWC, extents, poses, meta_data)
        -> (top_box, top_pose, top_target, top_weight, top_domain)
    _RoIPooling(pooled_height, pooled_width, spatial_scale)(features_NCHW, rois_Nx5)
        -> pooled (N, C, PH, PW)          rois: [batch, x1, y1, x2, y2]
    AverageDistanceLoss(num_classes, margin)(pred, target, weight, points, symmetry)
        -> loss (1,)
"""
import torch
from torch import nn

from .hough_voting_gpu_layer import hough_voting_gpu_op as hv
from .roi_pooling_layer import roi_pooling_op as rp
from .average_distance_loss import average_distance_loss_op as adl


class HoughVoting(nn.Module):
    def __init__(self, num_classes, threshold_vote, threshold_percentage, label_threshold=500, inlier_threshold=0.9,
                 skip_pixels=1, is_train=False):
        super().__init__()
        self.num_classes = int(num_classes)
        self.threshold_vote = float(threshold_vote)
        self.threshold_percentage = float(threshold_percentage)
        self.label_threshold = int(label_threshold)
        self.inlier_threshold = float(inlier_threshold)
        self.skip_pixels = int(skip_pixels)
        self.is_train = int(bool(is_train))

    def forward(self, label_2d, vertex_pred, extents, poses, meta_data):
        if vertex_pred.shape[-1] != 3 * self.num_classes:
            raise ValueError(f"vertex_pred must be NHWC with {3 * self.num_classes} channels")
        with torch.no_grad():  # the op's gradient is identically zero (hough_voting_gpu_op.cc:440-484)
            return hv.hough_voting_gpu(label_2d.to(torch.int32), vertex_pred, extents, meta_data, poses,
                                       self.is_train, self.threshold_vote, self.threshold_percentage,
                                       self.skip_pixels, inlier_threshold=self.inlier_threshold,
                                       label_threshold=self.label_threshold)


class _RoIPoolingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, rois, ph, pw, scale):
        top, arg = rp.roi_pool(features, rois, ph, pw, scale, 0, layout=1)  # NCHW, 5-column RoIs
        ctx.save_for_backward(features, rois, arg)
        ctx.params = (ph, pw, scale)
        return top

    @staticmethod
    def backward(ctx, grad):
        features, rois, arg = ctx.saved_tensors
        ph, pw, scale = ctx.params
        g = rp.roi_pool_grad(features, rois, arg, grad.contiguous(), ph, pw, scale, 0, layout=1)
        return g, None, None, None, None


class _RoIPooling(nn.Module):
    def __init__(self, pooled_height, pooled_width, spatial_scale):
        super().__init__()
        self.pooled_height = int(pooled_height)
        self.pooled_width = int(pooled_width)
        self.spatial_scale = float(spatial_scale)

    def forward(self, features, rois):
        if rois.dim() != 2 or rois.shape[1] != 5:
            raise ValueError("rois must be (N, 5): [batch, x1, y1, x2, y2]")
        return _RoIPoolingFn.apply(features.contiguous().float(), rois.contiguous().float(), self.pooled_height,
                                   self.pooled_width, self.spatial_scale)


class AverageDistanceLoss(nn.Module):
    def __init__(self, num_classes, margin=0.01):
        super().__init__()
        self.num_classes = int(num_classes)
        self.margin = float(margin)

    def forward(self, poses_pred, poses_target, poses_weight, points, symmetry):
        if poses_pred.shape[1] != 4 * self.num_classes:
            raise ValueError(f"poses_pred must have {4 * self.num_classes} columns")
        return adl.AverageDistanceFunction.apply(poses_pred, poses_target, poses_weight, points, symmetry,
                                                 self.margin)
