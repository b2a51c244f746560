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
                 "vst_plane_meanstd", "vst_simloss", "vst_simloss_bwd", "vst_resize_bilinear_bwd", "vst_upsample2x_bwd", "vst_copy_planes",
                 "vst_build_id"):
        assert name in protos, name
    assert protos["vst_conv_gemm"][0] == "int"
    assert len(protos["vst_conv_gemm"][1]) == 27
    # the C ABI is stateless: no global GEMM-mode setter; every GEMM / pack entry takes `mode`
    assert not [n for n in protos if "set_gemm_mode" in n or "get_gemm_mode" in n]
    for name in ("vst_pack_weight", "vst_conv_gemm", "vst_conv_gemm_padx", "vst_pack_weight_phase2", "vst_conv_dgrad_s2",
                 "vst_pack_weight_kwu", "vst_conv_dgrad_padout_kwu", "vst_conv_dgrad_padout", "vst_pack_weight_upsum",
                 "vst_conv_wgrad", "vst_conv_wgrad_rowsplit", "vst_gram", "vst_symmetrize", "vst_gemm_abt",
                 "vst_pack_matrix", "vst_attn_gemm"):
        assert protos[name][1][-2:] == ["int", "void*"], name


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libvst_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _lib.parse_header() if not hasattr(so, n)]
    assert not missing, missing
    lib = _lib.lib.load()
    # 400: round 4 (vst_adam_loss_scaled; round 3 added the `mask` argument of vst_fold_border /
    # vst_conv_dgrad_padout(_kwu) without a bump)
    assert lib.vst_version() == 400
    assert b"invalid" in lib.vst_strerror(-1)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libvst_hip.so not built")
def test_host_side_argument_validation_without_gpu():
    """Entry points validate arguments before touching the device: bad calls fail with VST_EINVAL."""
    lib = _lib.lib.load()
    assert lib.vst_conv_gemm(None, None, None, None, None, 1, 3, 8, 8, 4, 27, 8, 8, 3, 3, 0, 1, 1, 1, 0, 0, None, None,
                             None, 0, 0, None) == -1
    # split-K workspace is the caller's: a positive size with a NULL pointer is refused
    assert lib.vst_conv_gemm(1, 1, None, None, 1, 1, 16, 8, 8, 64, 144, 8, 8, 3, 3, 0, 1, 1, 1, 0, 0, None, None,
                             None, 1024, 19, None) == -1
    mp, kp = ctypes.c_int(), ctypes.c_int()
    assert lib.vst_conv_pack_dims(48, 243, ctypes.byref(mp), ctypes.byref(kp)) == 0
    assert (mp.value, kp.value) == (64, 256)
    assert lib.vst_conv_pack_dims(192, 1728, ctypes.byref(mp), ctypes.byref(kp)) == 0
    assert (mp.value, kp.value) == (192, 1728)
    assert lib.vst_wgrad_workspace(16, 192, 1728, 8192) > 0
    # GEMM arithmetic is a validated per-call argument: an unknown mode fails before any launch
    for bad in (-1, 5, 7, 8):
        assert lib.vst_pack_weight(1, 1, 4, 3, 3, 3, 0, 0, 64, 32, bad, None) == -1
        assert lib.vst_gemm_abt(1, 1, 1, 1, 1, 4, 4, 16, 1.0, bad, None) == -1
        assert lib.vst_conv_wgrad(1, 1, 1, 1, 1 << 20, 1, 3, 8, 8, 4, 8, 8, 3, 3, 0, 1, 1, 1, 0, bad, None) == -1
    # a workspace below both the halo slabs and the row-tiled kernel's need is refused before any
    # launch (ResidualBlock 192 -> 192 under bf16x6, whose halo slab exceeds the row-tiled workspace)
    geom = (2, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1, 1, 1)
    need = lib.vst_conv_wgrad_workspace(*geom, 3)
    rowtiled = lib.vst_wgrad_workspace(2, 192, 9 * 192, 64 * 128)
    assert need > 0 and rowtiled > 0
    n, cin, h, w, cout, ho, wo, kh, kw, gm, st, pd, up = geom
    small = min(need, rowtiled) - 1
    assert lib.vst_conv_wgrad(1, 1, 1, 1, small, n, cin, h, w, cout, ho, wo, kh, kw, gm, st, pd, up, 0, 3, None) == -1


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libvst_hip.so not built")
def test_build_provenance_matches_tree():
    """vst_build_id() (baked in by csrc/Makefile) equals the hash of this tree's csrc + header."""
    lib = _lib.lib.load()
    assert lib.vst_build_id().decode() == _lib.source_build_id()


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
