"""Flow datasets of the ReCoNet trainers with the per-item work on the GPU
(RC/datasets.py:42-281, RC/flowlib.py:34-64).

Drop-ins for `FlyingThings3D`, `Monkaa` and `FlyingThings3D_Monkaa` (same constructors, same
file indexing, same `(img1, img2, flow_into_past, mask)` items), plus `FramePairLoader`, the
batched replacement of `DataLoader(dataset, batch_size, shuffle=True)` (train_candy.py:34-39).

Split of the work:
  host   -- PNG/PGM decode (Pillow; the codec is not on the hot path), PFM header parse and raw
            payload read by the library's C reader (vst_pfm_read_header / vst_pfm_read) straight
            into pinned staging buffers, one non_blocking H2D copy per batch;
  device -- Pillow-exact bilinear resize + toTensor255 of every frame (vst_pil_resize_u8), the
            flow flipud / channel drop / bilinear resize / rescale (vst_flow_prep), the occlusion
            mask (vst_flow_warp_mask) and the motion-boundary mask multiplied in
            (vst_pil_resize_u8 mode 1).
Items come back as device tensors (the reference returns CPU tensors that the trainer moves
with `.to(device)`; the values are identical).  There is no CPU compute path.
"""
import os
import random
import threading
import ctypes

import numpy as np
import torch
from PIL import Image

from .. import ops
from .._lib import VstError, lib


def list_files(directory):
    """RC/utilities.py:23-25."""
    return sorted(f.path for f in os.scandir(directory) if f.is_file())


# ------------------------------------------------------------------------------- PFM (flowlib)
def pfm_header(path):
    """(width, height, channels, big_endian, payload offset, scale) of a PFM file; raises with
    readPFM's messages (RC/flowlib.py:40-58)."""
    w, h, c, be, off = (ctypes.c_int() for _ in range(5))
    scale = ctypes.c_float()
    rc = lib.load().vst_pfm_read_header(os.fsencode(path), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c),
                                        ctypes.byref(be), ctypes.byref(off), ctypes.addressof(scale))
    if rc != 0:
        raise Exception(lib.load().vst_strerror(rc).decode() + f" ({path})")
    return w.value, h.value, c.value, bool(be.value), off.value, scale.value


def read_pfm_raw(path, out=None):
    """Raw PFM payload as an (H, W, C) int32 array of float bits in file order (bottom-up rows),
    read by the C reader into `out` (e.g. a pinned staging slot) when given."""
    w, h, c, be, off, _ = pfm_header(path)
    if out is None:
        out = np.empty((h, w, c), np.int32)
    elif tuple(out.shape) != (h, w, c):
        raise VstError(f"{path}: PFM is {h}x{w}x{c}, staging slot is {tuple(out.shape)}")
    ptr = out.data_ptr() if isinstance(out, torch.Tensor) else out.ctypes.data
    rc = lib.load().vst_pfm_read(os.fsencode(path), ctypes.c_void_p(ptr), h * w * c * 4, off)
    if rc != 0:
        raise Exception(lib.load().vst_strerror(rc).decode() + f" ({path})")
    return out, be


def readPFM(file):  # noqa: N802 (flowlib's name)
    """flowlib.readPFM (RC/flowlib.py:34-64): (data flipped to top-down rows, scale)."""
    w, h, c, be, off, scale = pfm_header(file)
    raw, _ = read_pfm_raw(file)
    data = raw.view(">f4" if be else "<f4").reshape((h, w, 3) if c == 3 else (h, w))
    return np.flipud(data), scale


def read(file):
    """flowlib.read for the PFM flows the datasets use (RC/flowlib.py:14-22)."""
    if file.endswith(".pfm"):
        return readPFM(file)[0]
    raise Exception("don't know how to read %s" % file)


# ------------------------------------------------------------------------------- datasets
class _FlowDataset(torch.utils.data.Dataset):
    """Shared item / batch assembly for FlyingThings3D and Monkaa (RC/datasets.py:106-146)."""

    def __init__(self, resolution, frame_num, device=None):
        assert len(resolution) == 2 and isinstance(resolution, tuple), "Resolution must be a tuple of 2 integers."
        assert 1 <= frame_num and frame_num <= 9, "Frame number must be between 1 and 9."
        self.resolution = resolution
        self.frame_num = frame_num
        self.device = torch.device(device) if device is not None else None
        self.frame, self.flow, self.motion = [], [], []

    def __len__(self):
        return self.length

    def entries(self, idx):
        return self.frame[idx], self.flow[idx], self.motion[idx]

    def __getitem__(self, idx):
        _no_worker(type(self).__name__)
        img1, img2, flow, mask = prepare_batch([self.entries(idx)], self.resolution, self.frame_num, self.device)
        return img1[0], img2[0], flow[0], mask[0]


class FlyingThings3D(_FlowDataset):
    """RC/datasets.py:42-103 indexing: frames_finalpass/TRAIN/{A,B,C}/<seq>/left, flows
    optical_flow/TRAIN/.../into_{future,past}/left, motion_boundaries/TRAIN/.../into_future/left."""

    def __init__(self, path: str, resolution: tuple = (640, 360), frame_num: int = 1, device=None):
        super().__init__(resolution, frame_num, device)
        path_frame = os.path.join(path, "frames_finalpass/TRAIN")
        path_flow = os.path.join(path, "optical_flow/TRAIN")
        path_motion = os.path.join(path, "motion_boundaries/TRAIN")
        for p in (path_frame, path_flow, path_motion):
            assert os.path.exists(p), f"Path {p} does not exist."
        n = 10 - frame_num
        for abc in ["A", "B", "C"]:
            for folder in os.listdir(os.path.join(path_frame, abc)):
                files = list_files(os.path.join(path_frame, abc, folder, "left"))
                self.frame += [files[i:i + frame_num + 1] for i in range(n)]
        for abc in ["A", "B", "C"]:
            for folder in os.listdir(os.path.join(path_flow, abc)):
                fut = list_files(os.path.join(path_flow, abc, folder, "into_future", "left"))
                past = list_files(os.path.join(path_flow, abc, folder, "into_past", "left"))
                self.flow += [(fut[i + frame_num - 1], past[i + frame_num]) for i in range(n)]
        for abc in ["A", "B", "C"]:
            for folder in os.listdir(os.path.join(path_motion, abc)):
                files = list_files(os.path.join(path_motion, abc, folder, "into_future", "left"))
                self.motion += [files[i + frame_num] for i in range(n)]
        self.path = path
        self.length = len(self.frame)


class Monkaa(_FlowDataset):
    """RC/datasets.py:158-207 indexing: frames_finalpass/<seq>/left, optical_flow/<seq>/...,
    motion_boundaries/<seq>/into_future/left; every consecutive window of each sequence."""

    def __init__(self, path: str, resolution: tuple = (640, 360), frame_num: int = 1, device=None):
        super().__init__(resolution, frame_num, device)
        path_frame = os.path.join(path, "frames_finalpass")
        path_flow = os.path.join(path, "optical_flow")
        path_motion = os.path.join(path, "motion_boundaries")
        for p in (path_frame, path_flow, path_motion):
            assert os.path.exists(p), f"Path {p} does not exist."
        for folder in os.listdir(path_frame):
            files = list_files(os.path.join(path_frame, folder, "left"))
            self.frame += [files[i:i + frame_num + 1] for i in range(len(files) - frame_num)]
        for folder in os.listdir(path_flow):
            fut = list_files(os.path.join(path_flow, folder, "into_future", "left"))
            past = list_files(os.path.join(path_flow, folder, "into_past", "left"))
            self.flow += [(fut[i + frame_num - 1], past[i + frame_num]) for i in range(len(fut) - frame_num)]
        for folder in os.listdir(path_motion):
            files = list_files(os.path.join(path_motion, folder, "into_future", "left"))
            self.motion += [files[i + frame_num] for i in range(len(files) - frame_num)]
        self.path = path
        self.length = len(self.frame)


class FlyingThings3D_Monkaa(torch.utils.data.Dataset):  # noqa: N801 (reference name)
    """RC/datasets.py:256-281: Monkaa items first, then FlyingThings3D."""

    def __init__(self, path, resolution: tuple = (640, 360), frame_num: int = 1, device=None):
        if isinstance(path, str):
            self.monkaa = Monkaa(os.path.join(path, "monkaa"), resolution, frame_num, device)
            self.flyingthings3d = FlyingThings3D(os.path.join(path, "flyingthings3d"), resolution, frame_num, device)
        elif isinstance(path, list):
            self.monkaa = Monkaa(path[0], resolution, frame_num, device)
            self.flyingthings3d = FlyingThings3D(path[1], resolution, frame_num, device)
        else:
            raise ValueError("Path must be a string or a list of strings.")
        self.resolution, self.frame_num, self.device = resolution, frame_num, self.monkaa.device
        self.length = len(self.monkaa) + len(self.flyingthings3d)

    def __len__(self):
        return self.length

    def entries(self, idx):
        if idx < len(self.monkaa):
            return self.monkaa.entries(idx)
        return self.flyingthings3d.entries(idx - len(self.monkaa))

    def __getitem__(self, idx):
        if idx < len(self.monkaa):
            return self.monkaa[idx]
        return self.flyingthings3d[idx - len(self.monkaa)]


class Coco2014(torch.utils.data.Dataset):
    """RC/datasets.py:16-38: every file of <path>/train2014 (sorted), `Image.open(..).convert("RGB")
    .resize(resolution, Image.BILINEAR)` then toTensor255 -- the resize and conversion on the GPU
    (bit-exact with Pillow).  Items are (3, H, W) device tensors; `load_images` batches them."""

    def __init__(self, path: str, resolution: tuple = (256, 256), device=None):
        self.path = os.path.join(path, "train2014")
        self.resolution = resolution
        self.device = torch.device(device) if device is not None else None
        self.paths = list(list_files(self.path))
        self.length = len(self.paths)

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        _no_worker("Coco2014")
        return load_images([self.paths[idx]], self.resolution, self.device)[0]


def _no_worker(name):
    """Items are made by HIP kernels in the calling process; a forked DataLoader worker cannot use
    the GPU the parent already initialised, so say so instead of failing inside HIP."""
    if torch.utils.data.get_worker_info() is not None:
        raise VstError(f"{name} items are prepared on the GPU: iterate it with ImageLoader / FramePairLoader "
                       "(vst.reconet.datasets) instead of DataLoader(num_workers>0)")


def load_images(paths, resolution, device=None):
    """(len(paths), 3, H, W) fp32 = toTensor255(Image.open(p).convert("RGB").resize(resolution,
    BILINEAR)) per path; images sharing a source size go through one kernel launch."""
    return prepare_images(stage_images(paths), resolution, device)


def stage_images(paths):
    """Host half of load_images: decode into pinned uint8 staging, grouped by source size."""
    groups = {}
    for i, p in enumerate(paths):
        a = _decode(p, "RGB")
        groups.setdefault(a.shape, []).append((i, a))
    staged = []
    for shape, items in groups.items():
        host = torch.empty((len(items),) + shape, dtype=torch.uint8).pin_memory()
        for j, (_, a) in enumerate(items):
            host[j].numpy()[...] = a
        staged.append(([i for i, _ in items], host))
    return len(paths), staged


def prepare_images(staged, resolution, device=None):
    """Device half of load_images: one H2D copy + one resize launch per source size."""
    n, groups = staged
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    Wo, Ho = resolution
    out = torch.empty((n, 3, Ho, Wo), dtype=torch.float32, device=dev)
    for idx, host in groups:
        imgs = ops.pil_resize_to_tensor255(host.to(dev, non_blocking=True), resolution)
        out.index_copy_(0, torch.tensor(idx, device=dev), imgs)
    return out


# ------------------------------------------------------------------------------- batch assembly
def _decode(path, mode):
    img = Image.open(path)
    if mode == "RGB":
        img = img.convert("RGB")
    elif img.mode != "L":
        raise VstError(f"{path}: motion boundary image mode {img.mode!r}; the 8-bit path takes 'L'")
    return np.asarray(img)


def stage_batch(entries, frame_num):
    """Host half: decode / read every file of a batch into pinned staging tensors.
    Returns (frames (F+1, B, Hs, Ws, 3) u8, flows (2, B, Hf, Wf, C) int32 raw, big-endian flags,
    motion (B, Hm, Wm) u8); all items of a batch must share their source sizes."""
    B = len(entries)
    frames = flows = motion = None
    be = []
    for b, (fpaths, (ffut, fpast), mpath) in enumerate(entries):
        if len(fpaths) != frame_num + 1:
            raise VstError(f"item {b}: {len(fpaths)} frames for frame_num {frame_num}")
        for t, p in enumerate(fpaths):
            a = _decode(p, "RGB")
            if frames is None:
                frames = torch.empty((frame_num + 1, B) + a.shape, dtype=torch.uint8).pin_memory()
            if tuple(frames.shape[2:]) != a.shape:
                raise VstError(f"{p}: frame size {a.shape} differs from the batch's {tuple(frames.shape[2:])}")
            frames[t, b].numpy()[...] = a
        for k, p in enumerate((ffut, fpast)):
            w, h, c, big, _, _ = pfm_header(p)
            if flows is None:
                flows = torch.empty((2, B, h, w, c), dtype=torch.int32).pin_memory()
            read_pfm_raw(p, out=flows[k, b])
            be.append(big)
        m = _decode(mpath, "L")
        if motion is None:
            motion = torch.empty((B,) + m.shape, dtype=torch.uint8).pin_memory()
        if tuple(motion.shape[1:]) != m.shape:
            raise VstError(f"{mpath}: motion size {m.shape} differs from the batch's")
        motion[b].numpy()[...] = m
    if len(set(be)) > 1:
        raise VstError("a batch mixes little- and big-endian PFM files")
    return frames, flows, bool(be[0]), motion


def prepare_staged(staged, resolution, frame_num, device=None):
    """Device half: one H2D copy per staging tensor, then the prep kernels on the current stream."""
    frames, flows, big, motion = staged
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    T, B = frames.shape[:2]
    Wo, Ho = resolution
    fr = frames.to(dev, non_blocking=True)
    fl = flows.to(dev, non_blocking=True)
    mo = motion.to(dev, non_blocking=True)
    imgs = ops.pil_resize_to_tensor255(fr.view((T * B,) + tuple(fr.shape[2:])), resolution)
    imgs = imgs.view(T, B, 3, Ho, Wo)
    if frame_num == 1:
        img1, img2 = imgs[0], imgs[1]
    else:  # torch.cat(imgs[0:F], dim=0) per item: channel-stacked frames (a layout copy)
        img1 = imgs[:frame_num].permute(1, 0, 2, 3, 4).reshape(B, 3 * frame_num, Ho, Wo)
        img2 = imgs[1:].permute(1, 0, 2, 3, 4).reshape(B, 3 * frame_num, Ho, Wo)
    fl2 = ops.flow_prep(fl.view((2 * B,) + tuple(fl.shape[2:])), big, resolution)
    fut, past = fl2[:B], fl2[B:]
    mask = ops.flow_warp_mask(fut, past)
    ops.apply_motion_mask(mask, mo)
    return img1, img2, past, mask


def prepare_batch(entries, resolution, frame_num, device=None):
    """`default_collate([dataset[i] for i in batch])` of the reference, with the per-item work
    batched on the GPU: entries = [(frame paths, (flow_future, flow_past), motion path)]."""
    return prepare_staged(stage_batch(entries, frame_num), resolution, frame_num, device)


class _ShardedLoader:
    """Per-epoch seeded permutation shared by all ranks, padded by wrapping to a multiple of
    world_size (DistributedSampler semantics), each rank taking its strided share: every rank
    gets the same number of items and batches, so the per-step gradient all-reduce never waits on
    a rank that ran out of data."""

    def __init__(self, dataset, batch_size=1, shuffle=False, drop_last=False, seed=None, device=None, rank=None,
                 world_size=None):
        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        dist = torch.distributed
        on = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank() if on else 0)
        self.world_size = world_size if world_size is not None else (dist.get_world_size() if on else 1)
        if not 0 <= self.rank < self.world_size:
            raise VstError(f"rank {self.rank} outside world_size {self.world_size}")
        self.rng = random.Random(seed if seed is not None else 0 if self.world_size > 1 else None)
        self.device = device

    def _per_rank(self):
        n = len(self.dataset)
        return -(-n // self.world_size) if self.world_size > 1 else n

    def _indices(self):
        order = list(range(len(self.dataset)))
        if self.shuffle:
            self.rng.shuffle(order)
        if self.world_size > 1 and order:
            total = self._per_rank() * self.world_size
            while len(order) < total:  # wrap (repeats only the first items of the permutation)
                order += order[:total - len(order)]
        return order[self.rank::self.world_size]

    def __len__(self):
        n = self._per_rank()
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _index_batches(self):
        order = self._indices()
        for i in range(0, len(order), self.batch_size):
            idx = order[i:i + self.batch_size]
            if len(idx) < self.batch_size and self.drop_last:
                return
            yield idx


class ImageLoader(_ShardedLoader):
    """`DataLoader(Coco2014(...), batch_size, shuffle)` replacement (RC/train_single/
    train_coco2014.py:30-36): yields (B, 3, H, W) device batches made by `load_images` (Pillow-exact
    resize on the GPU, images sharing a source size in one launch); the host decode of the next
    batch runs in a background thread."""

    def __iter__(self):
        ds = self.dataset
        batches = ([ds.paths[j] for j in idx] for idx in self._index_batches())
        box = {}

        def stage(paths):
            try:
                box["staged"] = stage_images(paths)
            except BaseException as e:  # re-raised on the consumer side
                box["error"] = e

        yield from _prefetched(batches, stage, box, lambda st: prepare_images(st, ds.resolution, self.device))


def _prefetched(batches, stage, box, finish):
    nxt = next(batches, None)
    worker = None
    if nxt is not None:
        worker = threading.Thread(target=stage, args=(nxt,))
        worker.start()
    while worker is not None:
        worker.join()
        if "error" in box:
            raise box.pop("error")
        staged = box.pop("staged")
        nxt = next(batches, None)
        worker = None
        if nxt is not None:
            worker = threading.Thread(target=stage, args=(nxt,))
            worker.start()
        yield finish(staged)


class FramePairLoader(_ShardedLoader):
    """`DataLoader(dataset, batch_size, shuffle)` replacement (RC/train_single/train_candy.py:34-39):
    yields device batches `(img1, img2, flow_into_past, mask)`; the host decode / PFM read of the
    next batch runs in a background thread while the current batch is on the GPU.  rank /
    world_size (default: torch.distributed's when initialised): DP sharding as _ShardedLoader."""

    def _batches(self):
        for idx in self._index_batches():
            yield [self.dataset.entries(j) for j in idx]

    def __iter__(self):
        ds = self.dataset
        res, fn = ds.resolution, ds.frame_num
        box = {}

        def stage(entries):
            try:
                box["staged"] = stage_batch(entries, fn)
            except BaseException as e:  # re-raised on the consumer side
                box["error"] = e

        yield from _prefetched(self._batches(), stage, box, lambda st: prepare_staged(st, res, fn, self.device))
