"""CPU-side checks of the C-ABI boundary (no kernel launches without a GPU)."""
import ctypes
import os

import pytest

from vst import _lib


def test_header_parses_and_lists_entry_points():
    protos = _lib.parse_header()
    for name in ("vst_conv_gemm", "vst_conv_wgrad", "vst_gram", "vst_warp_fwd", "vst_warp_bwd", "vst_flow_warp_mask",
                 "vst_instnorm_fwd", "vst_instnorm_bwd", "vst_masked_sqdiff_fwd", "vst_adam", "vst_strerror",
                 # AdaAttN path
                 "vst_gemm_abt", "vst_pack_matrix", "vst_channel_norm", "vst_cos_attn_rows", "vst_cos_attn_rows_bwd",
                 "vst_softmax_rows", "vst_softmax_rows_bwd", "vst_adaattn_out", "vst_adaattn_out_bwd",
                 "vst_plane_meanstd", "vst_simloss", "vst_simloss_bwd", "vst_resize_bilinear_bwd", "vst_copy_planes",
                 "vst_set_gemm_mode", "vst_get_gemm_mode"):
        assert name in protos, name
    assert protos["vst_conv_gemm"][0] == "int"
    assert len(protos["vst_conv_gemm"][1]) == 24


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libvst_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _lib.parse_header() if not hasattr(so, n)]
    assert not missing, missing
    lib = _lib.lib.load()
    assert lib.vst_version() >= 100
    assert b"invalid" in lib.vst_strerror(-1)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libvst_hip.so not built")
def test_host_side_argument_validation_without_gpu():
    """Entry points validate arguments before touching the device: bad calls fail with VST_EINVAL."""
    lib = _lib.lib.load()
    assert lib.vst_conv_gemm(None, None, None, None, None, 1, 3, 8, 8, 4, 27, 8, 8, 3, 3, 0, 1, 1, 1, 0, 0, None, None,
                             None) == -1
    mp, kp = ctypes.c_int(), ctypes.c_int()
    assert lib.vst_conv_pack_dims(48, 243, ctypes.byref(mp), ctypes.byref(kp)) == 0
    assert (mp.value, kp.value) == (64, 256)
    assert lib.vst_conv_pack_dims(192, 1728, ctypes.byref(mp), ctypes.byref(kp)) == 0
    assert (mp.value, kp.value) == (192, 1728)
    assert lib.vst_wgrad_workspace(16, 192, 1728, 8192) > 0
    # GEMM arithmetic mode: host-side state, validated, default bf16x3 unless VST_GEMM_MODE says otherwise
    mode = lib.vst_get_gemm_mode()
    assert mode in (0, 1, 2)
    assert lib.vst_set_gemm_mode(7) == -1 and lib.vst_get_gemm_mode() == mode
    assert lib.vst_set_gemm_mode(0) == 0 and lib.vst_get_gemm_mode() == 0
    assert lib.vst_set_gemm_mode(mode) == 0


def test_product_fails_loudly_without_hip_tensors():
    import torch

    from vst import ops

    with pytest.raises(_lib.VstError):
        ops.conv2d(torch.zeros(1, 3, 8, 8), torch.zeros(4, 3, 3, 3), None, pad=1)


def test_adaattn_ops_fail_loudly_without_hip_tensors():
    import torch

    from vst.adaattn.attention import adaattn

    q = torch.zeros(1, 8, 2, 2)
    with pytest.raises(_lib.VstError):
        adaattn(q, q, q, q, "cosine")
