"""The ResidualBlock skip's gradient (RC/network.py:150 `out + residual`) is added inside conv1's data
gradient (ops.SkipGrad, vst_conv_dgrad_padout_accum) instead of by autograd.  The padded-grid
epilogue adds the interior straight onto the skip's gradient and the border fold adds the band, so
the interior is bitwise the separate sum (a + b is commutative) and the border band differs only in
the association of three fp32 terms."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("policy", ["bf16x6", "f32"])
@pytest.mark.parametrize("shape", [(2, 192, 16, 32), (3, 64, 20, 48), (1, 32, 9, 17)])
def test_dgrad_padout_accumulates(policy, shape):
    from vst import ops

    N, C, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(11)
    gz = torch.randn(N, C, H, W, device="cuda", generator=g)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05
    skip = torch.randn(N, C, H, W, device="cuda", generator=g)
    ops.gemm_role("fwd")
    saved = ops.POLICY_NAME[0]
    try:
        ops.use_policy(policy)
        ref = ops.conv_dgrad(gz, w, (N, C, H, W), 3, 1, 1, "reflect", 1) + skip
        acc = skip.clone()
        out = ops.conv_dgrad(gz, w, (N, C, H, W), 3, 1, 1, "reflect", 1, acc=acc)
        torch.cuda.synchronize()
    finally:
        ops.use_policy(saved)
    assert out.data_ptr() == acc.data_ptr()
    # interior (away from the 2-pixel band the fold touches): bitwise
    assert torch.equal(out[:, :, 2:-2, 2:-2], ref[:, :, 2:-2, 2:-2])
    err = ((out.double() - ref.double()).abs().max() / ref.abs().max()).item()
    assert err < 1e-6, err
    # against float64 autograd of pad -> conv (+ the skip)
    xd = torch.zeros(N, C, H, W, dtype=torch.float64, device="cuda", requires_grad=True)
    y = torch.nn.functional.conv2d(torch.nn.functional.pad(xd, (1, 1, 1, 1), mode="reflect"), w.double())
    y.backward(gz.double())
    exact = xd.grad + skip.double()
    rel = ((out.double() - exact).norm() / exact.norm()).item()
    assert rel < (2e-6 if policy == "f32" else 1e-5), rel


def test_reconet_step_skip_accum_on_off():
    """One train_candy step (RC/train_single/train_candy.py:77-152) with the skip accumulated in the
    data gradient and with autograd's sum: same losses, gradients and post-Adam parameters to fp32
    rounding of the band sums (bitwise-reproducible each way)."""
    from test_gpu_streams import _batch, _fresh_caches, _trainer
    from vst import ops

    ops.gemm_role("fwd")
    saved = (ops.SKIP_ACCUM, ops.POLICY_NAME[0])
    runs = []
    try:
        ops.use_policy("bf16x6")
        for on in (True, False, True):
            _fresh_caches()
            ops.SKIP_ACCUM = on
            tr = _trainer("reconet")
            out = tr.step(*_batch("reconet"))
            torch.cuda.synchronize()
            runs.append(({k: float(v) for k, v in out.items()}, tr.flat.g.clone()))
    finally:
        ops.SKIP_ACCUM = saved[0]
        ops.use_policy(saved[1])
    (l_on, g_on), (l_off, g_off), (l_on2, g_on2) = runs
    assert l_on == l_on2 and torch.equal(g_on, g_on2)
    for k in l_on:
        assert abs(l_on[k] - l_off[k]) <= 1e-6 * max(abs(l_off[k]), 1e-30), (k, l_on[k], l_off[k])
    rel = ((g_on.double() - g_off.double()).norm() / g_off.double().norm()).item()
    assert rel < 1e-5, rel
