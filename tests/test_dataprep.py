"""Flow-dataset frame-pair preparation (RC/datasets.py:42-281,
RC/flowlib.py:34-64) on the GPU.

Oracle: oracle/dataprep_ref.py, a numpy restatement of Pillow's 8-bit BILINEAR resampler and of
readPFM, pinned here bit-exactly against Pillow itself (the reference's dependency) and, through
the whole item, against the reference's own FlyingThings3D / Monkaa `__getitem__`
(tests/golden/dp_items.npz from tests/golden/gen_golden.py dataprep, over on-disk trees that
oracle/dataprep_ref.write_tree rebuilds bit-identically from a seed).

Tolerances: frames and motion masks are integer work -> bit-exact; flows are fp32 bilinear ->
1e-5 relative; the occlusion mask is a threshold of fp32 sums, so a pixel sitting on the threshold
may flip: at most 0.5% of mask pixels may differ (none did when written)."""

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import dataprep_ref as D
from oracle import reconet_ref as R

SHAPES = [(54, 96, 36, 64), (540, 960, 360, 640), (33, 47, 64, 90), (20, 20, 20, 13), (17, 31, 17, 31),
          (7, 9, 3, 2), (200, 400, 20, 30), (130, 70, 31, 17)]


def _rand_img(rng, H, W, C):
    if C == 3:
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    a = rng.integers(0, 256, (H, W), dtype=np.uint8)
    a[rng.random(a.shape) < 0.9] = 0
    return a


# ----------------------------------------------------------------------------- CPU: the oracle
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("C", [1, 3])
def test_oracle_resize_matches_pillow(shape, C):
    Hs, Ws, Ho, Wo = shape
    a = _rand_img(np.random.default_rng(Hs * 7 + C), Hs, Ws, C)
    ref = np.asarray(Image.fromarray(a).resize((Wo, Ho), Image.BILINEAR))
    np.testing.assert_array_equal(D.pil_resize_bilinear(a, (Wo, Ho)), ref)


@pytest.mark.parametrize("io", [(96, 64), (540, 360), (47, 90), (20, 20), (9, 2), (1, 5), (5, 1)])
def test_library_coeffs_match_oracle(io):
    """vst_pil_bilinear_coeffs is host code: callable without a GPU."""
    from vst import ops

    b, k = ops.pil_bilinear_coeffs(*io)
    rb, rk = D.pil_bilinear_coeffs(*io)
    np.testing.assert_array_equal(b, rb)
    np.testing.assert_array_equal(k, rk)


def test_library_pfm_reader(tmp_path):
    """The C PFM reader (host code) against readPFM's semantics, incl. big-endian and errors."""
    from vst.reconet import datasets as DS

    rng = np.random.default_rng(5)
    for le, color in ((True, True), (False, True), (True, False)):
        data = rng.standard_normal((7, 11, 3) if color else (7, 11)).astype(np.float32)
        p = str(tmp_path / f"f_{le}_{color}.pfm")
        D.write_pfm(p, data, scale=2.0, little_endian=le)
        ref, rs = D.read_pfm(p)
        got, gs = DS.readPFM(p)
        np.testing.assert_array_equal(np.asarray(got, np.float32), np.asarray(ref, np.float32))
        assert gs == rs == 2.0
        np.testing.assert_array_equal(np.asarray(ref, np.float32), data)
    bad = tmp_path / "bad.pfm"
    bad.write_bytes(b"P6\n3 2\n-1.0\n" + bytes(24))
    with pytest.raises(Exception, match="Not a PFM file."):
        DS.readPFM(str(bad))
    bad.write_bytes(b"PF\n3  2\n-1.0\n" + bytes(72))
    with pytest.raises(Exception, match="Malformed PFM header."):
        DS.readPFM(str(bad))
    bad.write_bytes(b"PF\n3 2\n-1.0\n" + bytes(70))
    with pytest.raises(Exception, match="does not match"):
        DS.readPFM(str(bad))


def _build(tmp_path, case):
    tag, kind, seed, H, W, folders, fpf, res, fn, items = case
    root = tmp_path / tag
    D.write_tree(str(root), kind, seed, H, W, folders, fpf)
    return str(root)


def _cases():
    # mirrors tests/golden/gen_golden.py DP_CASES (kept literal: gen_golden imports the reference)
    return (
        ("ft", "ft3d", 61, 36, 60, 1, 10, (40, 24), 1, (0, 4, 13, 26)),
        ("mk", "monkaa", 62, 20, 30, 2, 5, (48, 32), 2, (0, 2, 5)),
    )


def _golden_index(ds, root, g, tag, i):
    """Index of golden item i in `ds`: the reference (and the drop-in) order sequence folders by
    os.listdir, which is filesystem order, so items are matched by their first frame's path."""
    import os

    key = str(g[f"{tag}_{i}_key"])
    for j, entry in enumerate(ds.frame):
        if os.path.relpath(entry[0], root) == key:
            return j
    raise AssertionError(f"{key} not indexed")


def _oracle_item(ds, i):
    fpaths, (ffut, fpast), mpath = ds.entries(i)
    frames = [np.asarray(Image.open(p).convert("RGB")) for p in fpaths]
    fut = np.ascontiguousarray(D.read_pfm(ffut)[0])
    past = np.ascontiguousarray(D.read_pfm(fpast)[0])
    mot = np.asarray(Image.open(mpath))
    return D.getitem(frames, fut, past, mot, ds.resolution, R.flow_warp_mask)


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_oracle_items_match_reference(tmp_path, golden, case):
    """The oracle pipeline (and the drop-in's file indexing) against the reference's own items."""
    from vst.reconet import datasets as DS

    g = golden("dp_items")
    tag, kind, _, _, _, _, _, res, fn, items = case
    root = _build(tmp_path, case)
    cls = DS.FlyingThings3D if kind == "ft3d" else DS.Monkaa
    ds = cls(root, resolution=res, frame_num=fn)
    assert len(ds) == int(g[f"{tag}_len"])
    for i in items:
        img1, img2, flow, mask = _oracle_item(ds, _golden_index(ds, root, g, tag, i))
        np.testing.assert_array_equal(img1.numpy(), g[f"{tag}_{i}_img1"])
        np.testing.assert_array_equal(img2.numpy(), g[f"{tag}_{i}_img2"])
        np.testing.assert_allclose(flow.numpy(), g[f"{tag}_{i}_flow"], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(mask.numpy(), g[f"{tag}_{i}_mask"])


# ----------------------------------------------------------------------------- GPU: the kernels
@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_pil_resize_kernel_bit_exact(shape):
    from vst import ops

    Hs, Ws, Ho, Wo = shape
    rng = np.random.default_rng(Hs + Ws)
    imgs = np.stack([_rand_img(rng, Hs, Ws, 3) for _ in range(3)])
    got = ops.pil_resize_to_tensor255(torch.from_numpy(imgs).cuda(), (Wo, Ho)).cpu()
    for n in range(3):
        ref = D.to_tensor255(np.asarray(Image.fromarray(imgs[n]).resize((Wo, Ho), Image.BILINEAR)))
        assert torch.equal(got[n], ref)
    mot = np.stack([_rand_img(rng, Hs, Ws, 1) for _ in range(2)])
    base = torch.from_numpy((rng.random((2, Ho, Wo)) < 0.7).astype(np.float32))
    mask = ops.apply_motion_mask(base.clone().cuda(), torch.from_numpy(mot).cuda()).cpu()
    for n in range(2):
        m = np.asarray(Image.fromarray(mot[n]).resize((Wo, Ho), Image.BILINEAR))
        assert torch.equal(mask[n], base[n] * torch.from_numpy((m == 0).astype(np.float32)))


@pytest.mark.gpu
@pytest.mark.parametrize("big_endian", [False, True])
def test_flow_prep_kernel(big_endian):
    from vst import ops

    rng = np.random.default_rng(9 + big_endian)
    Hs, Ws, Ho, Wo = 27, 45, 36, 64
    flows = rng.standard_normal((3, Hs, Ws, 3)).astype(np.float32) * 4
    raw = np.flip(flows, axis=1).astype(">f4" if big_endian else "<f4")  # file order: bottom-up rows
    raw_bits = torch.from_numpy(np.ascontiguousarray(raw).view(np.int32))
    got = ops.flow_prep(raw_bits.cuda(), big_endian, (Wo, Ho)).cpu()
    for n in range(3):
        ref = D.flow_resize(flows[n], (Wo, Ho))
        torch.testing.assert_close(got[n], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_dataset_items_match_reference(tmp_path, golden, case):
    """Drop-in FlyingThings3D / Monkaa items on the GPU against the reference's own items."""
    from vst.reconet import datasets as DS

    g = golden("dp_items")
    tag, kind, _, _, _, _, _, res, fn, items = case
    root = _build(tmp_path, case)
    cls = DS.FlyingThings3D if kind == "ft3d" else DS.Monkaa
    ds = cls(root, resolution=res, frame_num=fn)
    flips = 0
    for i in items:
        img1, img2, flow, mask = (t.cpu() for t in ds[_golden_index(ds, root, g, tag, i)])
        assert img1.is_contiguous() or fn > 1
        np.testing.assert_array_equal(img1.numpy(), g[f"{tag}_{i}_img1"])
        np.testing.assert_array_equal(img2.numpy(), g[f"{tag}_{i}_img2"])
        np.testing.assert_allclose(flow.numpy(), g[f"{tag}_{i}_flow"], rtol=1e-5, atol=1e-5)
        flips += int((mask.numpy() != g[f"{tag}_{i}_mask"]).sum())
        assert flips <= 0.005 * mask.numel()
    # the batched loader yields the same items as the per-item path
    loader = DS.FramePairLoader(ds, batch_size=2, shuffle=False)
    b1, b2, bf, bm = next(iter(loader))
    for j in range(2):
        a1, a2, af, am = ds[j]
        assert torch.equal(b1[j], a1) and torch.equal(b2[j], a2)
        assert torch.equal(bf[j], af) and torch.equal(bm[j], am)
    assert len(loader) == (len(ds) + 1) // 2


@pytest.mark.gpu
def test_loader_feeds_training_step(tmp_path):
    """End to end: on-disk FlyingThings3D tree -> FramePairLoader (GPU prep) -> ReCoNetTrainer
    losses, against the oracle's items and the oracle's loss on them (1e-3 relative, the
    north-star fp32 tolerance), then one full optimiser step runs."""
    import oracle
    from oracle import shapes
    from vst.reconet import datasets as DS
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer
    from vst.synthetic import style_image

    root = str(tmp_path / "ft")
    D.write_tree(root, "ft3d", 71, 36, 60, 1, 10)
    ds = DS.FlyingThings3D(root, resolution=(64, 32), frame_num=1)
    batch = next(iter(DS.FramePairLoader(ds, batch_size=2)))
    P = oracle.seeded_params(shapes.reconet(), 5)
    VP = oracle.seeded_params(shapes.vgg16(), 6)
    model = N.ReCoNet()
    model.load_state_dict(P)
    vgg = N.Vgg16()
    vgg.load_state_dict(VP)
    style = style_image(8, 32, 64)
    tr = ReCoNetTrainer(model.cuda(), vgg.cuda(), style.cuda())
    img1, img2, flow, mask = batch
    out = tr.losses(torch.stack([img1, img2]), flow, mask)
    items = [_oracle_item(ds, j) for j in range(2)]
    o1, o2, of, om = (torch.stack([it[k] for it in items]) for k in range(4))
    assert torch.equal(img1.cpu(), o1) and torch.equal(img2.cpu(), o2)
    assert (mask.cpu() != om).float().mean() <= 0.005
    ref = R.reconet_losses(P, VP, o1, o2, of, om, R.style_grams(VP, style))
    for k in ("loss", "CL", "SL", "FTL", "OTL", "RL"):
        a, b = float(out[k].item()), float(ref[k])
        assert abs(a - b) <= 1e-3 * abs(b) + 1e-6, (k, a, b)
    res = tr.step(torch.stack([img1, img2]), flow, mask)
    assert torch.isfinite(res["loss"]).item()


def test_loader_rank_sharding(tmp_path):
    """FramePairLoader's DP sharding is host logic: disjoint, covering, seeded identically per rank."""
    from vst.reconet import datasets as DS

    root = str(tmp_path / "mk")
    D.write_tree(root, "monkaa", 3, 8, 8, 3, 6)
    ds = DS.Monkaa(root, resolution=(8, 8), frame_num=1)
    seen = []
    for r in range(3):
        ld = DS.FramePairLoader(ds, batch_size=2, shuffle=True, seed=11, rank=r, world_size=3)
        batches = list(ld._batches())
        assert len(batches) == len(ld)
        seen += [e[0][0] for b in batches for e in b]
    assert sorted(seen) == sorted(f[0] for f in ds.frame)
    with pytest.raises(Exception):
        DS.FramePairLoader(ds, rank=3, world_size=3)


@pytest.mark.parametrize("world", [2, 4])
def test_loader_shards_pad_to_equal_length(tmp_path, world):
    """len(dataset) % world != 0: the permutation is padded by wrapping (DistributedSampler), so
    every rank yields the same number of batches -- no rank blocks in the per-step all-reduce."""
    from vst.reconet import datasets as DS

    root = str(tmp_path / "mk")
    D.write_tree(root, "monkaa", 3, 8, 8, 1, 10)  # 9 items
    ds = DS.Monkaa(root, resolution=(8, 8), frame_num=1)
    assert len(ds) % world != 0
    for bs, drop in ((1, False), (2, False), (2, True)):
        lens, seen = set(), []
        for r in range(world):
            ld = DS.FramePairLoader(ds, batch_size=bs, shuffle=True, seed=5, rank=r, world_size=world, drop_last=drop)
            batches = list(ld._batches())
            assert len(batches) == len(ld)
            lens.add(len(batches))
            seen += [e[0][0] for b in batches for e in b]
        assert len(lens) == 1, lens
        if not drop:
            assert set(seen) == {f[0] for f in ds.frame}  # every item, a few twice
            assert len(seen) == -(-len(ds) // world) * world
    # the image loader shares the same sharding
    class Paths:
        paths = [f"p{i}" for i in range(7)]

        def __len__(self):
            return len(self.paths)

    n = {len(list(DS.ImageLoader(Paths(), batch_size=2, rank=r, world_size=world)._index_batches()))
         for r in range(world)}
    assert len(n) == 1


def test_dataset_items_refuse_dataloader_workers(tmp_path, monkeypatch):
    """The reference wraps its datasets in DataLoader(num_workers=4); items here are made by HIP
    kernels, which a forked worker cannot use -- a clear error names the replacement loaders."""
    import torch

    from vst.reconet import datasets as DS

    root = str(tmp_path / "mk")
    D.write_tree(root, "monkaa", 3, 8, 8, 1, 4)
    ds = DS.Monkaa(root, resolution=(8, 8), frame_num=1)
    monkeypatch.setattr(torch.utils.data, "get_worker_info", lambda: object())
    with pytest.raises(Exception, match="FramePairLoader"):
        ds[0]


def test_combined_dataset_indexing(tmp_path):
    """FlyingThings3D_Monkaa (RC/datasets.py:256-281): Monkaa items first, then FlyingThings3D;
    both path forms (root string, [monkaa, flyingthings3d] list)."""
    from vst.reconet import datasets as DS

    D.write_tree(str(tmp_path / "monkaa"), "monkaa", 1, 8, 8, 2, 4)
    D.write_tree(str(tmp_path / "flyingthings3d"), "ft3d", 2, 8, 8, 1, 10)
    for path in (str(tmp_path), [str(tmp_path / "monkaa"), str(tmp_path / "flyingthings3d")]):
        ds = DS.FlyingThings3D_Monkaa(path, resolution=(8, 8), frame_num=1)
        nm, nf = len(ds.monkaa), len(ds.flyingthings3d)
        assert (nm, nf) == (2 * 3, 3 * 9) and len(ds) == nm + nf
        assert ds.entries(0) == ds.monkaa.entries(0)
        assert ds.entries(nm) == ds.flyingthings3d.entries(0)
        assert ds.entries(len(ds) - 1) == ds.flyingthings3d.entries(nf - 1)
    with pytest.raises(ValueError):
        DS.FlyingThings3D_Monkaa(3)


def _coco(tmp_path, golden):
    import os

    from vst.reconet import datasets as DS

    g = golden("dp_items")
    root = str(tmp_path / "coco")
    D.write_coco(root, 63)
    ds = DS.Coco2014(root, resolution=(64, 48))
    assert len(ds) == int(g["coco_len"])
    for i in range(len(ds)):
        assert os.path.relpath(ds.paths[i], root) == str(g[f"coco_{i}_key"])  # sorted, like list_files
    return g, ds


def test_coco_oracle_matches_reference(tmp_path, golden):
    """Coco2014.__getitem__ (RC/datasets.py:35-38) restated: Pillow resample + toTensor255."""
    g, ds = _coco(tmp_path, golden)
    for i, p in enumerate(ds.paths):
        a = np.asarray(Image.open(p).convert("RGB"))
        got = D.to_tensor255(D.pil_resize_bilinear(a, ds.resolution)).numpy()
        np.testing.assert_array_equal(got, g[f"coco_{i}"])


@pytest.mark.gpu
def test_coco_items_match_reference(tmp_path, golden):
    from vst.reconet import datasets as DS

    g, ds = _coco(tmp_path, golden)
    for i in range(len(ds)):
        np.testing.assert_array_equal(ds[i].cpu().numpy(), g[f"coco_{i}"])
    batch = DS.load_images(ds.paths, ds.resolution).cpu().numpy()  # mixed sizes, grouped launches
    for i in range(len(ds)):
        np.testing.assert_array_equal(batch[i], g[f"coco_{i}"])


@pytest.mark.gpu
def test_image_loader_batches_match_reference(tmp_path, golden):
    """ImageLoader (the DataLoader(Coco2014) replacement of train_coco2014.py:30-36) yields the
    reference's items batched, bit-exact."""
    from vst.reconet import datasets as DS

    g, ds = _coco(tmp_path, golden)
    got = torch.cat(list(DS.ImageLoader(ds, batch_size=3))).cpu().numpy()
    assert got.shape[0] == len(ds)
    for i in range(len(ds)):
        np.testing.assert_array_equal(got[i], g[f"coco_{i}"])
