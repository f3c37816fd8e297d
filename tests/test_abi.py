"""The C-ABI boundary (include/posecnn_hip.h) on a CPU host: the library
loads, exports exactly the declared entry points with the declared arity,
and its host-side logic (versions, error strings, workspace sizing, argument
validation) answers without a GPU.  No compute call is made here."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "posecnn_hip.h")


def _declared():
    """{name: n_args} of every pcnn_* function declared in the header."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"\b(pcnn_\w+)\s*\(([^)]*)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


@pytest.fixture(scope="module")
def lib():
    from posecnn_amd import _lib, build
    if build.needs_build():
        build.build()
    return _lib.load()


def test_header_declares_the_reference_surface():
    names = set(_declared())
    # one entry per reference op launcher + the FC contraction
    for n in ("pcnn_hough_voting", "pcnn_hough_voting_grad", "pcnn_roi_pool_fwd", "pcnn_roi_pool_bwd",
              "pcnn_add_loss_fwd", "pcnn_add_loss_bwd", "pcnn_backproject_fwd", "pcnn_backproject_bwd",
              "pcnn_gemm", "pcnn_abi_version", "pcnn_strerror", "pcnn_box_nms", "pcnn_argmax_2d",
              "pcnn_hard_label_fwd", "pcnn_hard_label_bwd", "pcnn_hough_voting_prob", "pcnn_roi_pool_fwd_pair",
              "pcnn_hough_voting_compact", "pcnn_vertex_pred_compact"):
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    from posecnn_amd import _lib
    so = _lib.LIB_PATH
    nm = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    decl = _declared()
    missing = sorted(set(decl) - exported)
    assert not missing, f"declared but not exported: {missing}"
    # the Python binding covers the same set with the same arity
    assert set(_lib.exported_symbols()) == set(decl)
    for name, n in decl.items():
        assert len(_lib._SIGS[name][1]) == n, name
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr)


def test_version_and_errors(lib):
    assert lib.pcnn_abi_version() >= 1
    for code in (0, 1, 2, 3):
        assert lib.pcnn_strerror(code)
    assert lib.pcnn_strerror(999)


def test_workspace_sizing(lib):
    # Hough workspace grows with the batch and with the NMS (threshold_vote > 0) path
    a = lib.pcnn_hough_voting_workspace_size(1, 480, 640, 22, 10, -1.0)
    b = lib.pcnn_hough_voting_workspace_size(8, 480, 640, 22, 10, -1.0)
    c = lib.pcnn_hough_voting_workspace_size(1, 480, 640, 22, 10, 1.0)
    assert 0 < a < b and c > a
    assert lib.pcnn_roi_pool_bwd_workspace_size(8, 1152) > 0
    assert lib.pcnn_add_loss_workspace_size(1152, 22, 2620) >= 1152 * 4
    # GEMM: split-K slabs only when the tile count is small (both precisions);
    # the weight-gradient shapes run whole tiles
    assert lib.pcnn_gemm_workspace_size(1152, 4096, 25088, 1, 0) >= 2 * 1152 * 4096 * 4
    assert lib.pcnn_gemm_workspace_size(1152, 4096, 25088, 1, 1) >= 8 * 1152 * 4096 * 4
    assert lib.pcnn_gemm_workspace_size(1152, 4096, 25088, 1, 2) >= 8 * 1152 * 4096 * 4
    assert lib.pcnn_gemm_workspace_size(25088, 4096, 1152, 0, 1) == 256
    assert lib.pcnn_gemm_workspace_size(25088, 4096, 1152, 0, 2) == 256
    assert lib.pcnn_gemm_workspace_size(0, 4096, 25088, 0, 0) == 256


def test_argument_validation_without_gpu(lib):
    """Invalid arguments are rejected before any launch (PCNN_EINVAL = 1)."""
    nul = None
    # gemm: negative M; bad leading dimension; unknown precision
    assert lib.pcnn_gemm(-1, 4, 4, ctypes.c_void_p(16), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16), 4,
                         nul, 0, nul, 0, nul, nul, 0, nul, 0, nul) == 1
    assert lib.pcnn_gemm(4, 4, 8, ctypes.c_void_p(16), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16), 4,
                         nul, 0, nul, 0, nul, nul, 0, nul, 0, nul) == 1
    assert lib.pcnn_gemm(4, 4, 4, ctypes.c_void_p(16), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16), 4,
                         nul, 0, nul, 0, nul, nul, 7, nul, 0, nul) == 1
    # split-bf16 GEMM needs 16-B aligned operands
    assert lib.pcnn_gemm(4, 4, 4, ctypes.c_void_p(20), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16), 4,
                         nul, 0, nul, 0, nul, nul, 1, nul, 0, nul) == 1
    # gemm with dropout: keep_prob outside (0, 1]; drop pitch below N
    assert lib.pcnn_gemm_drop(4, 4, 4, ctypes.c_void_p(16), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16),
                              4, nul, 0, nul, 0, nul, 0, ctypes.c_float(0.0), nul, nul, 2, nul, 0, nul) == 1
    assert lib.pcnn_gemm_drop(4, 4, 4, ctypes.c_void_p(16), nul, 4, 0, ctypes.c_void_p(16), 4, 0, ctypes.c_void_p(16),
                              4, nul, 0, nul, 0, ctypes.c_void_p(16), 2, ctypes.c_float(0.5), nul, nul, 2, nul, 0,
                              nul) == 1
    # dropout masks: columns not a multiple of 4; keep_prob 0
    assert lib.pcnn_dropout_mask(ctypes.c_void_p(16), 4, 6, 8, nul, 1, nul, 0, ctypes.c_float(0.5), nul) == 1
    assert lib.pcnn_dropout_mask(ctypes.c_void_p(16), 4, 8, 8, nul, 1, nul, 0, ctypes.c_float(0.0), nul) == 1
    # roi pool: unknown layout
    assert lib.pcnn_roi_pool_fwd(ctypes.c_void_p(16), 1, 8, 8, 4, 7, ctypes.c_void_p(16), 1, 5, 0, nul, 1.0, 7, 7, 0,
                                 ctypes.c_void_p(16), ctypes.c_void_p(16), nul) == 1


def test_ops_fail_loudly_without_gpu():
    """No CPU fallback: the op layer refuses to run without a HIP device."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from posecnn_amd import _lib
    from posecnn_amd.roi_pooling_layer import roi_pooling_op as rp
    with pytest.raises(_lib.PcnnError):
        rp.roi_pool(torch.zeros(1, 8, 8, 4), torch.zeros(1, 7), 7, 7, 1.0, 0)
