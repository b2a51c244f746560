"""Drop-in for RT/utilities.py: put this directory first on sys.path (the reference's train.py does
`from utilities import ...`).  Implementation: vst.rtnstv.utilities (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.rtnstv.utilities import *  # noqa: E402,F401,F403
from vst.rtnstv.utilities import flow_warp_mask, gram_matrix, vgg_normalize, warp  # noqa: E402,F401
