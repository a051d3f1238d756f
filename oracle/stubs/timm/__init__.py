"""Oracle-only stand-in for timm (imported by the reference but unused on the detector path, block.py:1723)."""
