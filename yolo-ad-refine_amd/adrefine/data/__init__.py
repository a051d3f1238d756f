"""Training-data side of the hot path: the v8 augmentation chain with its pixel work on the GPU (augment.py)."""
