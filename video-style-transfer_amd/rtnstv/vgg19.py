"""Drop-in for RT/vgg19.py: put this directory first on sys.path (the reference's train.py does
`from vgg19 import ...`).  Implementation: vst.rtnstv.vgg19 (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.rtnstv.vgg19 import *  # noqa: E402,F401,F403
from vst.rtnstv.vgg19 import VGG19  # noqa: E402,F401
