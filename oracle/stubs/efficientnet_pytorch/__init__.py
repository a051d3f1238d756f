"""Oracle-only stand-in (imported by attention.py, not on the detector path)."""
