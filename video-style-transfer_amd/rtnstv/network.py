"""Drop-in for RT/network.py: put this directory first on sys.path (the reference's train.py does
`from network import ...`).  Implementation: vst.rtnstv.network (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.rtnstv.network import *  # noqa: E402,F401,F403
from vst.rtnstv.network import Conv, Deconv, Res, StylizingNetwork  # noqa: E402,F401
