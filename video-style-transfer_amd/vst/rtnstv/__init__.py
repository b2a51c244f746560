"""MI355X RTNSTV path: drop-in `network` / `vgg19` / `utilities` modules
and the RT/train.py training step, on the same HIP kernels as ReCoNet plus ConvTranspose2d,
the sqrt-TV regulariser and the tanh image output."""
