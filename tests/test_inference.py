"""ReCoNet inference path (RC/utilities.py:108-235): `Inference`,
`calculate_mse` and `cvframe_to_tensor` on the HIP frame kernels, against golden vectors made by
running the reference's own Inference / calculate_mse (tests/golden/gen_golden.py gen_infer:
trained SD2 checkpoint shipped with the reference, and a seeded 2-frame-window SD2).

Tolerances: the frame conversion kernels are bit-exact (uint8 and fp32); stylised uint8 frames
come from fp32 forwards whose rounding differs from the CPU's, so a pixel whose value sits at an
integer boundary may truncate one lower/higher: |diff| <= 1 everywhere and <= 1% of bytes
differing; calculate_mse within 1e-3 relative (fp32 contract of north_star)."""
import numpy as np
import pytest
import torch

import oracle
from oracle import reconet_ref as R
from oracle import shapes
from vst.synthetic import video_frames


def _ckpt(golden, tag):
    g = golden("rc_infer")
    if tag == "a":
        ck = golden("rc_sd_ckpt")
        return {k.split("/", 1)[1]: torch.from_numpy(v) for k, v in ck.items() if k.startswith("ReCoNetSD2/")}
    spec = shapes.reconet_sd2(2)
    return {k: v.detach() for k, v in oracle.seeded_params(spec, int(g["b_ckpt_seed"])).items()}


def _case(golden, tag):
    g = golden("rc_infer")
    seed, T, ff, n = (int(v) for v in g[f"{tag}_meta"])
    return g, video_frames(seed, T), (None if ff < 0 else ff), n


@pytest.mark.parametrize("tag", ["a", "b"])
def test_oracle_inference_matches_reference(golden, tag):
    """Pins the oracle's restatement against the reference's own outputs."""
    g, frames, ff, n = _case(golden, tag)
    P = _ckpt(golden, tag)
    outs = R.inference(R.reconet_sd2_forward, P, frames, n, ff)
    assert len(outs) == int(g[f"{tag}_n_out"])
    d = np.abs(outs[0].astype(int) - g[f"{tag}_frame0"].astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-2
    for i, o in enumerate(outs):
        d = np.abs(o[:48].astype(int) - g[f"{tag}_rows"][i].astype(int))
        assert d.max() <= 1
    mse = R.calculate_mse(R.reconet_sd2_forward, P, frames, n)
    assert abs(mse - float(g[f"{tag}_mse"])) <= 1e-4 * abs(float(g[f"{tag}_mse"]))


@pytest.mark.gpu
def test_frame_kernels_bit_exact():
    from vst import ops

    rng = np.random.default_rng(7)
    for N, H, W in ((3, 36, 64), (2, 7, 9)):  # vector (HW % 4 == 0) and scalar kernels
        f = rng.integers(0, 256, size=(N, H, W, 3), dtype=np.uint8)
        t = ops.frames_to_tensor(torch.from_numpy(f).cuda()).cpu()
        ref = torch.stack([R.cvframe_to_tensor(x) for x in f])
        assert torch.equal(t, ref)
        y = torch.from_numpy(rng.uniform(-40, 300, size=(N, 3, H, W)).astype(np.float32))
        y[0, 0, 0, :3] = torch.tensor([255.0, 0.0, 254.99998])
        cl = torch.empty_like(y).cuda()
        u8 = ops.tensor_to_frames(y.cuda(), clamped=cl).cpu().numpy()
        yc = y.clamp(0, 255)
        assert torch.equal(cl.cpu(), yc)
        ref = np.ascontiguousarray(yc.permute(0, 2, 3, 1).numpy()[..., ::-1]).astype(np.uint8)
        assert np.array_equal(u8, ref)
    x = [torch.from_numpy(rng.uniform(0, 255, (1, 3, 36, 64)).astype(np.float32)) for _ in range(4)]
    out = torch.zeros(1, device="cuda")
    ops.frame_diff_mse(*(v.cuda() for v in x), out)
    ref = torch.nn.functional.mse_loss(x[1] - x[0], x[3] - x[2]).item()
    assert abs(out.item() - ref) <= 1e-6 * ref


@pytest.mark.gpu
@pytest.mark.parametrize("tag,batch", [("a", 1), ("a", 3), ("b", 1), ("b", 2)])
def test_inference_golden(golden, tag, batch, tmp_path):
    from vst.reconet import network as N
    from vst.reconet.inference import Inference, calculate_mse

    g, frames, ff, n = _case(golden, tag)
    path = str(tmp_path / "m.pth")
    torch.save(_ckpt(golden, tag), path)
    outs = list(Inference(N.ReCoNetSD2, n, path, frames, "cuda", ff, batch_frames=batch))
    assert len(outs) == int(g[f"{tag}_n_out"])
    assert outs[0].shape == (360, 640, 3) and outs[0].dtype == np.uint8
    d = np.abs(outs[0].astype(int) - g[f"{tag}_frame0"].astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-2, (d.max(), (d > 0).mean())
    for i, o in enumerate(outs):
        d = np.abs(o[:48].astype(int) - g[f"{tag}_rows"][i].astype(int))
        assert d.max() <= 1
        s = o.reshape(-1, 3).astype(np.int64).sum(0)
        assert np.all(np.abs(s - g[f"{tag}_sums"][i]) <= 0.01 * 360 * 640)
    mse = calculate_mse(N.ReCoNetSD2, n, path, frames, "cuda", batch_frames=batch)
    assert abs(mse - float(g[f"{tag}_mse"])) <= 1e-3 * abs(float(g[f"{tag}_mse"]))


@pytest.mark.gpu
def test_cvframe_to_tensor_and_short_video():
    from vst.reconet import network as N
    from vst.reconet.inference import Inference, cvframe_to_tensor

    f = video_frames(3, 1)[0]
    t = cvframe_to_tensor(f)
    assert t.is_cuda and torch.equal(t.cpu(), R.cvframe_to_tensor(f))
    sd = N.ReCoNetSD2(3).state_dict()
    with pytest.raises(ValueError):
        Inference(N.ReCoNetSD2, 3, sd, video_frames(3, 2), "cuda")
