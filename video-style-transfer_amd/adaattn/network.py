"""Drop-in for AA/network.py: put this directory first on sys.path (the reference's trainers do
`from network import ...`).  Implementation: vst.adaattn.network (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.adaattn.network import AdaAttN, AdaAttnNoConv, Conv, ConvReLU, ConvReluInterpolate, ConvTanh, CosineSimilarity, Decoder, Softmax, StylizingNetwork  # noqa: E402,F401
