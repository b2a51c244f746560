"""Synthetic frame-pair batches: identical for the HIP path, the oracle and
the CPU baseline because everything random comes from numpy PCG64 with a caller-given seed.

A batch mirrors what `FlyingThings3D_Monkaa.__getitem__` yields
(`RC/datasets.py:100-146`): `(img1, img2, flow_into_past, mask)` with frames in [0, 255),
a smooth optical flow (coarse U(-8, 8) px field at 1/16 resolution, bilinearly upsampled) and
`mask = flow_warp_mask(flow_into_future, flow_into_past) * motion` where `motion` is a
Bernoulli(0.9) stand-in for the motion-boundary image.  `mask_fn(flo01, flo10)` is injected so
the product path can use its HIP `flow_warp_mask` and tests can use the oracle's.
"""
import numpy as np
import torch
import torch.nn.functional as F


def _smooth(rng, B, H, W, coarse=None, amp=8.0, jitter=None):
    hc, wc = max(1, H // 16), max(1, W // 16)
    c = rng.uniform(-amp, amp, (B, 2, hc, wc)) if coarse is None else -coarse + rng.uniform(-jitter, jitter, coarse.shape)
    full = F.interpolate(torch.from_numpy(c.astype(np.float32)), size=(H, W), mode="bilinear", align_corners=False)
    return c, full


def frame_pair_parts(seed, B, H, W):
    """The random draws of one batch (CPU tensors): img1, img2, flow into the future, flow into the
    past, motion mask -- the occlusion mask is formed from them by frame_pair_batch's mask_fn."""
    rng = np.random.default_rng(seed)
    img1 = torch.from_numpy(rng.uniform(0.0, 255.0, (B, 3, H, W)).astype(np.float32))
    img2 = torch.from_numpy(rng.uniform(0.0, 255.0, (B, 3, H, W)).astype(np.float32))
    fwd_c, flow_future = _smooth(rng, B, H, W)
    _, flow_past = _smooth(rng, B, H, W, coarse=fwd_c, jitter=1.0)
    motion = torch.from_numpy((rng.random((B, H, W)) < 0.9).astype(np.float32))
    return img1, img2, flow_future, flow_past, motion


def frame_pair_batch(seed, B, H, W, mask_fn=None, device="cpu"):
    parts = frame_pair_parts(seed, B, H, W)
    img1, img2, flow_future, flow_past, motion = (t.to(device) for t in parts)
    if mask_fn is None:
        mask = motion
    else:
        mask = torch.stack([mask_fn(flow_future[b], flow_past[b]) for b in range(B)]) * motion
    return img1, img2, flow_past.contiguous(), mask.contiguous()


def style_image(seed, H, W, device="cpu"):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.uniform(0.0, 255.0, (1, 3, H, W)).astype(np.float32)).to(device)


def content_style_batch(seed, B, H, W, device="cpu"):
    """(content1, content2, style) images in [0, 255) as `VidevoWikiArt` yields them
    (AA/datasets.py), B per tensor."""
    rng = np.random.default_rng(seed)
    out = [torch.from_numpy(rng.uniform(0.0, 255.0, (B, 3, H, W)).astype(np.float32)).to(device) for _ in range(3)]
    return tuple(out)


def video_frames(seed, T, H=360, W=640, step=3):
    """Synthetic cv2-style clip for the inference path: T x H x W x 3 uint8 BGR frames, frame t
    the window [t*step, t*step + W) of one seeded noise strip (a horizontal pan)."""
    rng = np.random.default_rng(seed)
    strip = rng.integers(0, 256, size=(H, W + step * max(T - 1, 0), 3), dtype=np.uint8)
    return np.stack([strip[:, t * step:t * step + W] for t in range(T)])
