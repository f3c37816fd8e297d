"""The TensorFlow custom-op binding (tf_ops/posecnn_tf_ops.cc) -- CPU only.

TensorFlow is not in this image, so the library itself is not built here
(tf_ops/build_tf_ops.py skips); the source is compiled with -fsyntax-only
against a stub of the TF op API subset it uses (tests/tf_stub: not
TensorFlow), and its registrations are checked against the reference's op
interface (op names, attrs, inputs, outputs: hough_voting_gpu_op.cc:37-60,
roi_pooling_op.cc:29-50, average_distance_loss_op.cc:38-54,
backprojecting_op.cc:30-53) as restated below."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tf_ops", "posecnn_tf_ops.cc")

# op -> (attrs, inputs, outputs) of the reference registrations
OPS = {
    "Houghvotinggpu": (["T: {float, double}", "is_train: int", "threshold_vote: float", "threshold_percentage: float",
                        "skip_pixels: int"],
                       ["bottom_label: int32", "bottom_vertex: T", "bottom_extents: T", "bottom_meta_data: T",
                        "bottom_gt: T"],
                       ["top_box: T", "top_pose: T", "top_target: T", "top_weight: T", "top_domain: int32"]),
    "HoughvotinggpuGrad": (["T: {float, double}"], ["bottom_label: int32", "bottom_vertex: T", "grad: T"],
                           ["output_label: T", "output_vertex: T"]),
    "RoiPool": (["T: {float, double}", "pooled_height: int", "pooled_width: int", "spatial_scale: float",
                 "pool_channel: int"], ["bottom_data: T", "bottom_rois: T"], ["top_data: T", "argmax: int32"]),
    "RoiPoolGrad": (["T: {float, double}", "pooled_height: int", "pooled_width: int", "spatial_scale: float",
                     "pool_channel: int"], ["bottom_data: T", "bottom_rois: T", "argmax: int32", "grad: T"],
                    ["output: T"]),
    "Averagedistance": (["T: {float, double}", "margin: float"],
                        ["bottom_prediction: T", "bottom_target: T", "bottom_weight: T", "bottom_point: T",
                         "bottom_symmetry: T"], ["loss: T", "bottom_diff: T"]),
    "AveragedistanceGrad": (["T: {float, double}", "margin: float"], ["bottom_diff: T", "grad: T"], ["output: T"]),
    "Backproject": (["T: {float, double}", "grid_size: int", "kernel_size: int", "threshold: float"],
                    ["bottom_data: T", "bottom_label: T", "bottom_depth: T", "bottom_meta_data: T",
                     "bottom_label_3d: T"], ["top_data: T", "top_label: T", "top_flag: T"]),
    "BackprojectGrad": (["T: {float, double}", "grid_size: int", "kernel_size: int", "threshold: float"],
                        ["bottom_data: T", "bottom_depth: T", "bottom_meta_data: T", "grad: T"], ["output: T"]),
}


def test_registrations_match_reference_interface():
    src = open(SRC).read()
    for op, (attrs, ins, outs) in OPS.items():
        m = re.search(r'REGISTER_OP\("%s"\)(.*?);' % op, src, re.S)
        assert m, op
        body = m.group(1)
        assert re.findall(r'\.Attr\("([^"]+)"\)', body) == attrs, op
        assert re.findall(r'\.Input\("([^"]+)"\)', body) == ins, op
        assert re.findall(r'\.Output\("([^"]+)"\)', body) == outs, op
        assert re.search(r'REGISTER_KERNEL_BUILDER\(Name\("%s"\)\.Device\(DEVICE_GPU\)' % op, src), op


def test_compiles_against_op_api_stub():
    cc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(cc):
        pytest.skip("hipcc not present")
    subprocess.check_call([cc, "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "tf_stub"), "-I",
                           os.path.join(ROOT, "include"), SRC])


def test_build_skips_without_tensorflow():
    try:
        import tensorflow  # noqa: F401
        pytest.skip("TensorFlow present: the library builds")
    except ImportError:
        pass
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tf_ops"))
    import build_tf_ops
    assert build_tf_ops.build(verbose=False) is None
