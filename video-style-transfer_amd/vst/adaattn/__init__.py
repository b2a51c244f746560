"""AdaAttN (AA/*) video-training path on HIP kernels."""
