"""MI355X ReCoNet video inference: drop-in for `Inference`, `calculate_mse` and
`cvframe_to_tensor` of RC/utilities.py:108-235.

Per frame the reference runs: cv2 BGR uint8 frame -> `toTensor255` (ToTensor, mul 255) -> model
forward under no_grad -> `clamp(0, 255)` -> HWC -> RGB2BGR -> `astype(uint8)`, and (for
calculate_mse) `MSELoss(mean)(x_t1 - x_t, y_t1 - y_t)` of consecutive content/stylised frames
with one `.item()` per frame.  Here every step of that chain runs on the GPU:
  * frames are read on the host in chunks of `batch_frames`, staged in one pinned uint8 buffer
    and uploaded with one async copy (3 bytes per pixel instead of 12 as fp32);
  * `vst_frames_to_tensor` turns the uint8 BGR chunk into fp32 RGB planes (bit-identical to
    ToTensor*255), `vst_tensor_to_frames` does clamp + BGR + truncation into uint8 in one pass;
  * the stylizer runs its HIP conv/IN kernels on `batch_frames` windows at once (frames are
    independent samples of the forward; each window is `input_frame_num` consecutive frames
    concatenated on channels, as the reference's `torch.cat(imgs, dim=0)`);
  * calculate_mse writes each pair's MSE into a device slot (`vst_frame_diff_mse`) and syncs
    once at the end, then sums the float32 values left to right in double precision like the
    reference's `loss += mse(x, y).item()`.
`video_path` may be a file path (opened with cv2.VideoCapture, so cv2 must be importable -- it
is not in this image) or, as an extension, a uint8 array (T,H,W,3) / iterable of cv2-style BGR
frames.  Frames that are not 360x640 are resized by cv2 on the host exactly as the reference
does (RC/utilities.py:120-122); without cv2 they raise.
"""
import numpy as np
import torch

from .. import ops

FRAME_HW = (360, 640)  # RC/utilities.py:121: cv2.resize(frame, (640, 360))


def _cv2():
    try:
        import cv2  # noqa: PLC0415
    except ImportError as e:  # pragma: no cover - cv2 is absent in this image
        raise ImportError("reading video files / resizing frames needs OpenCV (cv2), as the reference does") from e
    return cv2


class _FrameSource:
    """cv2.VideoCapture-like reader: `.read() -> (ret, frame)` over a path or in-memory frames."""

    def __init__(self, video):
        if isinstance(video, (str, bytes)) or hasattr(video, "__fspath__"):
            self._cap = _cv2().VideoCapture(str(video))
            self._it = None
        else:
            self._cap = None
            self._it = iter(video)

    def read(self):
        if self._cap is not None:
            return self._cap.read()
        try:
            return True, next(self._it)
        except StopIteration:
            return False, None

    def release(self):
        if self._cap is not None:
            self._cap.release()


def _host_frame(frame):
    """RC/utilities.py:119-122 host part: check / resize to 360x640 (cv2 INTER_LINEAR)."""
    if frame is None:
        raise ValueError("the video has fewer frames than input_frame_num / first_frame need")
    frame = np.asarray(frame)
    if frame.dtype != np.uint8 or frame.ndim != 3 or frame.shape[2] != 3:
        raise ValueError(f"frames must be HxWx3 uint8 (cv2 BGR), got {frame.dtype} {frame.shape}")
    if frame.shape[:2] != FRAME_HW:
        cv2 = _cv2()
        frame = cv2.resize(frame, (FRAME_HW[1], FRAME_HW[0]), interpolation=cv2.INTER_LINEAR)
    return np.ascontiguousarray(frame)


def cvframe_to_tensor(frame, device="cuda"):
    """RC/utilities.py:118-123: cv2 BGR uint8 frame -> (3,360,640) fp32 RGB in [0,255], computed
    by the HIP kernel on `device` (the reference returns a CPU tensor that callers `.to(device)`)."""
    f = torch.from_numpy(_host_frame(frame)).to(device)
    return ops.frames_to_tensor(f.unsqueeze(0))[0]


def _load_model(model_class, input_frame_num, model_path, device):
    model = model_class(input_frame_num).to(device)
    sd = model_path if isinstance(model_path, dict) else torch.load(model_path, weights_only=True, map_location=device)
    model.load_state_dict(sd, strict=True)
    return model


class _Stream:
    """Chunked frame pipeline shared by Inference and calculate_mse: keeps the last
    `n - 1` device frames and produces (windows, newest content frames) per chunk."""

    def __init__(self, reader, n, device, batch_frames):
        self.reader, self.n, self.device, self.B = reader, n, device, max(1, int(batch_frames))
        self.pinned = None
        self.history = None  # (n-1, 3, H, W) device frames preceding the next chunk
        self.eof = False

    def _upload(self, frames):
        k = len(frames)
        H, W = frames[0].shape[:2]
        shape = (max(self.B, self.n), H, W, 3)
        if self.pinned is None or tuple(self.pinned.shape) != shape:
            self.pinned = torch.empty(shape, dtype=torch.uint8, pin_memory=True)
        host = self.pinned[:k].numpy()
        for i, f in enumerate(frames):
            host[i] = f
        dev = self.pinned[:k].to(self.device, non_blocking=True)
        out = ops.frames_to_tensor(dev)
        # the pinned buffer is reused by the next chunk: wait for this copy first
        torch.cuda.current_stream().synchronize()
        return out

    def first(self, first_frame):
        """RC/utilities.py:196-206: skip to first_frame, read input_frame_num frames."""
        n = self.n
        if first_frame is None or first_frame < n:
            first_frame = n
        for _ in range(first_frame - n):
            self.reader.read()
        frames = [_host_frame(self.reader.read()[1]) for _ in range(n)]
        return self._upload(frames)  # (n, 3, H, W)

    def chunks(self, initial):
        """Yields (windows (b, 3n, H, W), content (b, 3, H, W)) until the video ends."""
        n = self.n
        all_frames = initial
        while True:
            k = all_frames.shape[0] - (n - 1)  # windows available
            _, _, H, W = all_frames.shape
            if n == 1:
                windows = all_frames
            else:
                windows = torch.stack([all_frames[i:i + n].reshape(3 * n, H, W) for i in range(k)])
            yield windows, all_frames[n - 1:]
            if self.eof:
                return
            self.history = all_frames[all_frames.shape[0] - (n - 1):] if n > 1 else None
            new = []
            while len(new) < self.B:
                ret, frame = self.reader.read()
                if not ret:
                    self.eof = True
                    break
                new.append(_host_frame(frame))
            if not new:
                return
            up = self._upload(new)
            all_frames = torch.cat([self.history, up]) if n > 1 else up


class Inference:
    """RC/utilities.py:179-235: iterate a video, yielding stylised HxWx3 uint8 BGR frames.
    `batch_frames` (extension, default 1 = the reference's schedule) runs that many
    consecutive windows per forward."""

    def __init__(self, model_class, input_frame_num, model_path, video_path, device="cuda", first_frame=None,
                 batch_frames=1):
        self.model = _load_model(model_class, input_frame_num, model_path, device)
        self.video_path = video_path
        self.input_frame_num = input_frame_num
        self.device = device
        self.cap = _FrameSource(video_path)
        self._stream = _Stream(self.cap, input_frame_num, device, batch_frames)
        self._initial = self._stream.first(first_frame)
        self.imgs = list(self._initial.unbind(0))

    def __del__(self):
        cap = getattr(self, "cap", None)
        if cap is not None:
            cap.release()

    def __iter__(self):
        host = None
        for windows, _ in self._stream.chunks(self._initial):
            with torch.no_grad():
                *_, out = self.model(windows)
                frames = ops.tensor_to_frames(out)
            if host is None or host.shape[0] < frames.shape[0] or host.shape[1:] != frames.shape[1:]:
                host = torch.empty(tuple(frames.shape), dtype=torch.uint8, pin_memory=True)
            h = host[:frames.shape[0]]
            h.copy_(frames)
            for img in h.numpy():
                yield img.copy()


def calculate_mse(model_class, input_frame_num, model_path, video_path, device="cuda", batch_frames=1):
    """RC/utilities.py:126-176: mean over consecutive frame pairs of
    MSELoss(mean)((x_t1 - x_t), (y_t1 - y_t)), y = clamp(model(window), 0, 255)."""
    model = _load_model(model_class, input_frame_num, model_path, device)
    cap = _FrameSource(video_path)
    try:
        st = _Stream(cap, input_frame_num, device, batch_frames)
        initial = st.first(None)
        slots = []
        prev_x = prev_y = None
        for windows, content in st.chunks(initial):
            with torch.no_grad():
                *_, out = model(windows)
            y = torch.empty_like(out)
            ops.tensor_to_frames(out, clamped=y)
            for b in range(y.shape[0]):
                x_t1, y_t1 = content[b:b + 1], y[b:b + 1]
                if prev_x is not None:
                    slot = torch.empty(1, dtype=torch.float32, device=y.device)
                    ops.frame_diff_mse(prev_x, x_t1, prev_y, y_t1, slot)
                    slots.append(slot)
                prev_x, prev_y = x_t1, y_t1
    finally:
        cap.release()
    vals = torch.cat(slots).cpu().tolist() if slots else []
    loss = 0
    for v in vals:
        loss += v
    return loss / len(vals)
