"""Drop-in for RC/flowlib.py's PFM reader (`read`, `readPFM`), parsed by the library's C reader.
Implementation: vst.reconet.datasets."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.reconet.datasets import read, readPFM  # noqa: E402,F401
