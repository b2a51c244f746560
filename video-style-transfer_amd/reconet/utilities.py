"""Drop-in for the hot-path helpers of RC/utilities.py (`warp`, `flow_warp_mask`, `gram_matrix`,
`vgg_normalize`) and of its inference helpers (`Inference`, `calculate_mse`,
`cvframe_to_tensor`).  Implementation: vst.reconet.utilities (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.reconet.utilities import flow_warp_mask, gram_matrix, vgg_normalize, warp  # noqa: E402,F401
from vst.reconet.inference import Inference, calculate_mse, cvframe_to_tensor  # noqa: E402,F401
