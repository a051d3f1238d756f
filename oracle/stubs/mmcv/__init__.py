"""Oracle-only stand-in for mmcv (absent from this image, unpinned in the reference).
Only ModulatedDeformConv2d (mmcv.ops) and build_norm_layer (mmcv.cnn) are used on the path
(reference head.py:749-782)."""
__version__ = "0.0.0-oracle-stub"
