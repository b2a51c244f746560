"""MI355X ReCoNet path: drop-in `network` / `utilities` modules and the training step."""
