"""Drop-in for RC/network.py: put this directory first on sys.path (the reference's trainers do
`from network import ReCoNet, Vgg16`).  Implementation: vst.reconet.network (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.reconet.network import *  # noqa: E402,F401,F403
from vst.reconet.network import (ConvInstRelu, ConvLayer, ConvTanh, ReCoNet, ReCoNetSD1, ReCoNetSD2,  # noqa: E402,F401
                                 ResidualBlock, SelectiveLoadModule, UpsampleConvInstRelu, UpsampleConvLayer, Vgg16)
