"""Drop-in for AA/lossfn.py: put this directory first on sys.path (the reference's trainers do
`from lossfn import ...`).  Implementation: vst.adaattn.lossfn (HIP kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vst.adaattn.lossfn import cosine_distance, global_stylized_loss, image_similarity_loss, local_feature_loss  # noqa: E402,F401
