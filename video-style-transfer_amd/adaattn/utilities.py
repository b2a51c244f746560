"""Drop-in for the hot-path helpers of AA/utilities.py: put this directory first on sys.path (the reference's trainers do
`from utilities import ...`).  Implementation: vst.adaattn.utilities (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.adaattn.utilities import feature_down_sample, flow_warp_mask, vgg_normalize, warp  # noqa: E402,F401
