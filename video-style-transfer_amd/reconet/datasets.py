"""Drop-in for RC/datasets.py's datasets (`Coco2014`, `FlyingThings3D`, `Monkaa`,
`FlyingThings3D_Monkaa`) with the per-item resize / flow / mask work on the GPU, plus the
batched `FramePairLoader`.  Implementation: vst.reconet.datasets (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.reconet.datasets import (  # noqa: E402,F401
    Coco2014, FlyingThings3D, FlyingThings3D_Monkaa, FramePairLoader, Monkaa, list_files, load_images, prepare_batch)
