"""ctypes binding of libvst_hip.so (the C ABI declared in include/vst_hip.h).

The argument types of every entry point are read from the header itself, so the header is the
single source of truth for the boundary.  There is no CPU fallback: if the shared library is
missing or fails to load, every op raises.
"""
import ctypes
import glob
import hashlib
import os
import re

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# VST_LIB_PATH: a library built from THIS tree's sources with other compile-time choices (csrc/Makefile
# VARIANT_FLAGS), for A/B step measurements only (tools/gpu_r04_*.sh); its build id must still match
# the sources here, so it can never be a stale or foreign build
LIB_PATH = os.environ.get("VST_LIB_PATH") or os.path.join(_HERE, "libvst_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "vst_hip.h")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")


def source_build_id(csrc=CSRC, header=HEADER_PATH):
    """sha256 (first 16 hex digits) over the sorted csrc/*.hip, *.h and Makefile, then the public
    header: the recipe csrc/Makefile bakes into vst_build_id() at build time."""
    files = sorted(os.path.basename(f) for pat in ("*.hip", "*.h", "Makefile") for f in glob.glob(os.path.join(csrc, pat)))
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    with open(header, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]

_CTYPES = {
    "int": ctypes.c_int,
    "long": ctypes.c_long,
    "float": ctypes.c_float,
    "void": None,
    "void*": ctypes.c_void_p,
    "float*": ctypes.c_void_p,
    "int*": ctypes.POINTER(ctypes.c_int),
    "char*": ctypes.c_char_p,
}


def parse_header(path=HEADER_PATH):
    """{name: (restype, [argtypes])} for every `extern "C"` prototype in the header."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"^\s*((?:const\s+)?\w+\s*\**)\s*(vst_\w+)\s*\(([^)]*)\)\s*;", text, flags=re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3)

        def norm(t):
            t = t.replace("const", "").strip()
            base = re.sub(r"\s+", "", t)
            return base

        rt = norm(ret)
        argts = []
        if args.strip() not in ("", "void"):
            for a in args.split(","):
                a = a.strip()
                a = re.sub(r"\b\w+$", "", a) if not a.endswith("*") else a
                argts.append(norm(a))
        protos[name] = (rt, argts)
    return protos


class VstError(RuntimeError):
    pass


class _Lib:
    def __init__(self):
        self._lib = None

    def load(self):
        if self._lib is not None:
            return self._lib
        if not os.path.exists(LIB_PATH):
            raise VstError(f"libvst_hip.so not built ({LIB_PATH}); run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (rt, argts) in parse_header().items():
            fn = getattr(lib, name)
            fn.restype = _CTYPES[rt] if rt != "char*" else ctypes.c_char_p
            fn.argtypes = [_CTYPES[a] for a in argts]
        # provenance: the library must have been built from the sources of this tree
        built = lib.vst_build_id().decode()
        want = source_build_id() if os.path.isdir(CSRC) else built
        if built != want:
            raise VstError(f"libvst_hip.so build id {built} does not match the sources in {CSRC} ({want}): "
                           "stale build, rebuild with `make -C video-style-transfer_amd/csrc`")
        self.build_id = built
        self._lib = lib
        return lib

    def __getattr__(self, name):
        fn = getattr(self.load(), name)

        def call(*args):
            rc = fn(*args)
            if fn.restype is ctypes.c_int and rc != 0:
                msg = self.load().vst_strerror(rc).decode()
                raise VstError(f"{name} failed: {msg} (rc={rc})")
            return rc

        return call


lib = _Lib()


def ptr(t):
    """Device pointer of a contiguous fp32 CUDA tensor (or None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise VstError("vst ops need HIP (cuda) tensors; there is no CPU path")
    if t.dtype != torch.float32:
        raise VstError(f"vst ops compute in fp32, got {t.dtype}")
    if not t.is_contiguous():
        raise VstError("vst ops need contiguous NCHW tensors")
    return t.data_ptr()


def ptr_rows(t):
    """(device pointer, batch stride) of a tensor whose per-sample slices t[n] are contiguous
    (e.g. a channel slice of a concat buffer); the batch stride may exceed t[0].numel()."""
    if not t.is_cuda or t.dtype != torch.float32:
        raise VstError("vst ops need fp32 HIP (cuda) tensors; there is no CPU path")
    if not t[0].is_contiguous():
        raise VstError("vst ops need per-sample contiguous tensors")
    return t.data_ptr(), t.stride(0)


def stream():
    return torch.cuda.current_stream().cuda_stream
