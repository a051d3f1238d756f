"""adrefine — MI355X-native (gfx950) hot path of the YOLO-AD-Refine detector.

Host side mirrors the reference's operator API for this path (module class names, constructor signatures,
parameter names / state_dict keys, yaml `parse_model` rules, head output contract, v8DetectionLoss and
non_max_suppression). All arithmetic runs in hand-written HIP kernels in `lib/libadr_hip.so`, called
through its C ABI (include/adr.h). There is no CPU or eager fallback: if the library is missing or no GPU is
present, the ops raise.
"""
import torch  # noqa: F401  (torch's HIP runtime first: libadr_hip.so then binds to that one, not a second copy)

from . import native  # noqa: F401  (loads libadr_hip.so eagerly, fails loudly)

__version__ = "0.1.0"
