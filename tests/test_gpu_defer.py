"""Deferred, batched parameter-gradient reductions (kernels.py WgradDeferral: adr_dotsum_batched,
adr_nc_reduce_batched, adr_gn_param_grad_batched) against the immediate per-call path: one bf16 training
forward/backward of the 701 graph at 320^2 bs 2 with each ADR_DEFER_* switch off, the gradient arena compared
bitwise with the default (all deferred). Covers the AYHead's per-level shared GroupNorm modules (a repeated
destination starts a new batched launch) and flushes with more entries than one launch holds; and the grouped
WGRAD partial launches (adr_conv2d_wgrad_partials_batched) against one launch per conv."""
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _arena():
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    from gpu_util import load_recipe_into
    from recipe import synthetic_images, synthetic_labels
    torch.manual_seed(0)
    m = DetectionModel(str(CFG), compute_dtype=torch.bfloat16)
    load_recipe_into(m)
    m = m.cuda()
    tr = FusedTrainer(m, batch_size=2)
    b = {"img": synthetic_images(2, 320, seed=5).cuda(), **synthetic_labels(2, 80, seed=6)}
    tr.forward_backward(b)
    torch.cuda.synchronize()
    return tr.grad.clone()


@pytest.mark.parametrize("knob", ["_DEFER_DOT", "_DEFER_COLSUM", "_DEFER_GN", "_DEFER_WGRAD", "all"])
def test_deferred_reductions_bitwise(knob):
    """_DEFER_WGRAD: the WGRAD partials of the stage's convs grouped into one launch per tile shape at the flush
    (adr_conv2d_wgrad_partials_batched) — the same tiles / splits per conv, so bitwise the per-conv launches."""
    import adrefine.kernels as K
    names = ["_DEFER_DOT", "_DEFER_COLSUM", "_DEFER_GN", "_DEFER_WGRAD"] if knob == "all" else [knob]
    ref = _arena()
    saved = {n: getattr(K, n) for n in names}
    try:
        for n in names:
            setattr(K, n, False)
        got = _arena()
    finally:
        for n, v in saved.items():
            setattr(K, n, v)
    assert bool(torch.isfinite(ref).all()) and float(ref.abs().max()) > 0
    diff = (ref != got).nonzero().numel()
    assert torch.equal(ref, got), f"{diff} arena entries differ with {names} off"
