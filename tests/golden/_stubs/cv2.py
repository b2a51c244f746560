"""Empty stand-in for OpenCV (absent in this image); only imported, never called, on the path."""
INTER_LINEAR = 1
