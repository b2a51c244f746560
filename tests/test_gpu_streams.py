"""The side streams (weight gradients and input-only loss targets on a second HIP
stream) change WHERE work runs, never what it computes.  The first training step of a fresh process
is the one that races if an ordering is missing (the lazily created constants of the AdaAttN modules,
the shared packs of the frozen loss networks are filled on whichever stream touches them first), so
every run here starts from emptied caches.  The HIP step has no float atomics on any gradient
(the warp and image-similarity adjoints gather in a fixed order), so the same step with the side
streams on and off -- and on again -- must give BITWISE equal loss terms, flat gradients and
post-Adam parameters (ReCoNet train_candy step, RC/train_single/train_candy.py:77-152; AdaAttN
train_video step, AA/train_video.py:78-122, under the fp32-class and the fp16 policy)."""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _fresh_caches():
    from vst import ops
    from vst.adaattn import attention

    ops._PACK_CACHE.clear()
    ops._CONST_FILL.clear()
    ops._SEED.clear()
    attention._ONES.clear()
    attention._AFFINE_ID.clear()


def _trainer(kind):
    import oracle
    from oracle import shapes

    def seeded(m, spec, seed):
        P = oracle.seeded_params(spec, seed)
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.copy_(P[n])
        return m.cuda()

    if kind == "reconet":
        from vst.reconet.network import ReCoNet, Vgg16
        from vst.reconet.train import ReCoNetTrainer
        from vst.synthetic import style_image

        return ReCoNetTrainer(seeded(ReCoNet(), shapes.reconet(), 1), seeded(Vgg16(), shapes.vgg16(), 2),
                              style_image(3, 64, 128).cuda())
    from vst.adaattn.network import StylizingNetwork
    from vst.adaattn.train import AdaAttNTrainer
    from vst.adaattn.vgg19 import VGG19

    return AdaAttNTrainer(seeded(StylizingNetwork("cosine"), shapes.stylizing_network(), 1),
                          seeded(VGG19(), shapes.vgg19(), 2), activation="cosine")


def _batch(kind):
    from vst.synthetic import content_style_batch, frame_pair_batch

    if kind == "reconet":
        from oracle import reconet_ref as R

        img1, img2, flow, mask = frame_pair_batch(1234, 2, 64, 128, mask_fn=R.flow_warp_mask)
        return torch.stack([img1, img2]).cuda(), flow.cuda(), mask.cuda()
    c1, c2, s = content_style_batch(1234, 2, 64, 128)
    return (torch.stack([c1, c2, s]).cuda(),)


@pytest.mark.parametrize("kind,policy", [("reconet", "bf16x6"), ("adaattn", "bf16x6"), ("adaattn", "f16")])
def test_side_streams_bitwise(kind, policy):
    from vst import ops

    ops.gemm_role("fwd")  # (applies the environment's policy first, so it is the one restored)
    saved = (ops.WGRAD_SIDE, ops.CONTENT_SIDE, ops.POLICY_NAME[0])
    runs = []
    try:
        ops.use_policy(policy)
        for side in (True, False, True):
            _fresh_caches()
            ops.WGRAD_SIDE = ops.CONTENT_SIDE = side
            tr = _trainer(kind)
            out = tr.step(*_batch(kind))
            torch.cuda.synchronize()
            runs.append(({k: float(v) for k, v in out.items()}, tr.flat.g.clone(), tr.flat.p.clone()))
    finally:
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = saved[:2]
        ops.use_policy(saved[2])
    (l0, g0, p0) = runs[0]
    assert torch.isfinite(g0).all()
    assert float(g0.abs().max()) > 0
    for i, (l, g, p) in enumerate(runs[1:], 1):
        assert l == l0, (i, l, l0)
        assert torch.equal(g, g0), (i, float((g - g0).abs().max() / g0.abs().max()))
        assert torch.equal(p, p0), i


@contextlib.contextmanager
def _poisoned_allocations():
    """Every float HIP tensor made through torch.empty (the library's outputs, workspaces, packs and
    constants) is filled with NaN on the allocating stream first: a read of memory before its
    producer wrote it -- on another stream that skipped a wait -- then shows as a NaN instead of
    silently reading what an earlier run left in a recycled block."""
    orig = torch.empty

    def empty(*a, **k):
        t = orig(*a, **k)
        if t.is_cuda and t.is_floating_point():
            t.fill_(float("nan"))
        return t

    torch.empty = empty
    try:
        yield
    finally:
        torch.empty = orig


# vst_test_delay iterations (~3.5 us each): 1500 ~ 5 ms, far longer than any kernel of these steps
_DELAY = 1500
_PLACES = ("side_branch", "wgrad_side", "pack", "persistent")


def _run(kind, side, places=(), poison=False):
    from vst import ops

    _fresh_caches()
    ops.WGRAD_SIDE = ops.CONTENT_SIDE = side
    ops.TEST_DELAY.clear()
    ops.TEST_DELAY.update({p: _DELAY for p in places})
    try:
        with _poisoned_allocations() if poison else contextlib.nullcontext():
            tr = _trainer(kind)
            out = tr.step(*_batch(kind))
            torch.cuda.synchronize()
    finally:
        ops.TEST_DELAY.clear()
    return {k: float(v) for k, v in out.items()}, tr.flat.g.clone(), tr.flat.p.clone()


@pytest.mark.parametrize("kind,policy", [("reconet", "bf16x6"), ("adaattn", "f16")])
def test_side_streams_delay_injected(kind, policy):
    """Each cross-stream hand-off of the step widened by a 5 ms stall on the stream at that point
    (vst_test_delay): the head of the input-only side branch (its reads of the main stream's data
    features start late), the head of each side-stream weight gradient (its reads of gz / x start
    late, the join before Adam is tested against a late writer), each weight pack kernel (a reader on
    the other stream that skipped the pack's event would run first), each lazily created constant's
    fill (ditto for constant()) -- one placement at a time, then all four, every allocation poisoned
    with NaN.  Each run must equal, bitwise, the step with the side streams off, no stalls and no
    poison (which itself must equal the poisoned in-line step: no kernel reads memory it did not
    write)."""
    from vst import ops

    ops.gemm_role("fwd")
    saved = (ops.WGRAD_SIDE, ops.CONTENT_SIDE, ops.POLICY_NAME[0])
    try:
        ops.use_policy(policy)
        ref = _run(kind, False)
        cases = [("inline-poisoned", False, (), True)]
        cases += [(p, True, (p,), True) for p in _PLACES]
        cases += [("all", True, _PLACES, True)]
        bad = []
        for name, side, places, poison in cases:
            l, g, p = _run(kind, side, places, poison)
            if not (l == ref[0] and torch.equal(g, ref[1]) and torch.equal(p, ref[2])):
                gd = float((g - ref[1]).abs().max() / ref[1].abs().max())
                bad.append((name, {k: l[k] - ref[0][k] for k in l}, gd))
    finally:
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = saved[:2]
        ops.use_policy(saved[2])
    assert not bad, bad


@pytest.mark.parametrize("kind,policy", [("reconet", "bf16x6"), ("adaattn", "f16")])
def test_step_bitwise_under_scratch_poison(kind, policy):
    """Kernels with register spills keep them in per-wave private (scratch) slots that the next
    dispatch on the same queue reuses.  A kernel that read a private slot before writing it would pick
    up whatever the previous kernel left there -- in a repeated step usually the same bits, which hides
    it.  vst_test_scratch_poison fills every scratch slot of both streams with NaN first (three slot
    sizes up to 4.5 KB per lane, 4096 x 256 lanes each); the step must still equal, bitwise, the step
    run without the poison (the one-off f16 difference of round 5 came from a
    build whose spilling conv tile held 576 B of private memory per lane)."""
    from vst import ops
    from vst._lib import lib

    ops.gemm_role("fwd")
    saved = (ops.WGRAD_SIDE, ops.CONTENT_SIDE, ops.POLICY_NAME[0])
    try:
        ops.use_policy(policy)
        ref = _run(kind, True)
        dev = torch.device("cuda")
        for st in (torch.cuda.current_stream(dev), ops._side_stream(dev)):
            lib.vst_test_scratch_poison(4096, float("nan"), st.cuda_stream)
        torch.cuda.synchronize()
        l, g, p = _run(kind, True)
    finally:
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = saved[:2]
        ops.use_policy(saved[2])
    assert l == ref[0], (l, ref[0])
    assert torch.equal(g, ref[1]) and torch.equal(p, ref[2])


def test_warp_backward_deterministic_under_converging_flow():
    """The warp adjoint's per-source-pixel lists (CSR, sorted by output pixel before the sum) give
    bitwise identical gradients run after run, also where many taps converge on one source pixel (a
    flow that folds a whole row band onto a few pixels: long lists take the queued block sort), and
    match the scatter form in float64 (RC/utilities.py:39-57 backward)."""
    from vst import ops

    g = torch.Generator().manual_seed(7)
    B, C, H, W = 2, 5, 24, 40
    x = torch.randn(B, C, H, W, generator=g)
    flo = torch.randn(B, 2, H, W, generator=g) * 3
    # converging band: columns 10..29 of rows 5..14 all point at (x=20, y=10)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    band = (yy >= 5) & (yy < 15) & (xx >= 10) & (xx < 30)
    flo[:, 0][:, band] = (20.3 - xx[band])
    flo[:, 1][:, band] = (10.6 - yy[band])
    gout = torch.randn(B, C, H, W, generator=g)
    xd, fd, gd = x.cuda().requires_grad_(True), flo.cuda(), gout.cuda()
    outs = []
    for _ in range(4):
        xd.grad = None
        ops.warp(xd, fd).backward(gd)
        torch.cuda.synchronize()
        outs.append(xd.grad.clone())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    x64 = x.double().requires_grad_(True)
    Hf, Wf = float(H - 1), float(W - 1)
    grid = torch.stack([(xx + flo[:, 0].double()) * 2 / Wf - 1, (yy + flo[:, 1].double()) * 2 / Hf - 1], dim=-1)
    y = torch.nn.functional.grid_sample(x64, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
    y.backward(gout.double())
    err = float((outs[0].cpu().double() - x64.grad).abs().max() / x64.grad.abs().max())
    assert err < 1e-5, err
