"""Build tf_ops/posecnn_tf_ops.so: the reference's TensorFlow op names
(Houghvotinggpu, RoiPool, Averagedistance, Backproject and their gradients)
on the C-ABI of posecnn_amd/libposecnn_hip.so.

Only when TensorFlow-ROCm is importable (it is not in this image: the script
then reports the skip and exits 0).  The reference side loads the library in
its op modules, e.g. lib/hough_voting_gpu_layer/hough_voting_gpu_op.py:
    _module = tf.load_op_library('<repo>/tf_ops/posecnn_tf_ops.so')
    hough_voting_gpu = _module.hough_voting_gpu
(INTEGRATION.md §2)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def build(verbose=True):
    try:
        import tensorflow as tf
    except ImportError:
        if verbose:
            print("tf_ops: TensorFlow not importable; TF custom-op library not built", file=sys.stderr)
        return None
    sys.path.insert(0, ROOT)
    from posecnn_amd import build as pb
    lib = pb.build(verbose=verbose)
    out = os.path.join(HERE, "posecnn_tf_ops.so")
    cmd = (["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-shared", "-fPIC", os.path.join(HERE, "posecnn_tf_ops.cc"),
            "-I", os.path.join(ROOT, "include"), "-o", out]
           + tf.sysconfig.get_compile_flags() + tf.sysconfig.get_link_flags()
           + ["-L", os.path.dirname(lib), "-lposecnn_hip", "-Wl,-rpath," + os.path.dirname(lib)])
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    build()
