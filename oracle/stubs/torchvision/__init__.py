"""Oracle-only stand-in for torchvision (absent from this image). Only `torchvision.ops.nms` is on the
reference's hot path (utils/ops.py:292); it is restated in torchvision/ops/__init__.py."""
__version__ = "0.25.0"
from . import ops  # noqa: E402,F401
