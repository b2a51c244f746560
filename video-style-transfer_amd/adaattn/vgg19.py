"""Drop-in for AA/vgg19.py: put this directory first on sys.path (the reference's trainers do
`from vgg19 import ...`).  Implementation: vst.adaattn.vgg19 (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.adaattn.vgg19 import VGG19  # noqa: E402,F401
