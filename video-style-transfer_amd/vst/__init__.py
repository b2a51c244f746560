"""vst — MI355X-native (gfx950) video-style-transfer training hot path.

Host side mirrors the reference's module API (vst.reconet.network, vst.reconet.utilities); all
compute runs in libvst_hip.so (C ABI: include/vst_hip.h).  Importing this package does not touch
the GPU or load the library; the first op does, and fails loudly if the library is missing.
"""
__version__ = "0.1.0"
