"""Oracle-only stand-in for OpenCV: the reference imports cv2 at module load (utils/__init__.py:22)
but nothing on the detector's compute path calls it. Constants resolve to 0; functions are no-ops."""
__version__ = "0.0.0-oracle-stub"


def setNumThreads(n):  # noqa: N802 (OpenCV naming)
    return None


def __getattr__(name):
    return 0
