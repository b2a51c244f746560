"""Offline stand-in for the parts of torchvision the reference imports at module top.

Container-only test infrastructure for `tests/golden/gen_golden.py`: torchvision is not
installed in this image and pretrained weights cannot be fetched, so this package supplies
architecture-only `models.vgg16/vgg19` (standard "D"/"E" feature configs, weights are
overwritten by the generator with seeded values) and the handful of `transforms` objects
constructed at import time by the reference's `utilities.py` files.
"""
from . import models, transforms  # noqa: F401
