"""Staged backward (the DDP bucket stages, engine/ddp.py) against the unstaged one on one GPU: fp32 parity mode, the
701 graph at 320^2 bs 2, cuts that detach a layer output read later by several layers through an index (not -1:
L13 -> L16 / L18, L19 -> L20 / L28, L20 -> L23 / L25) as well as the bucket-derived default. The gradient arena
must agree to fp32 rounding (the stage split changes only the order in which fan-out gradients are summed)."""
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _arena(stages):
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    from gpu_util import load_recipe_into
    from recipe import synthetic_images, synthetic_labels
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    m = m.cuda()
    tr = FusedTrainer(m, batch_size=2, stages=stages)
    b = {"img": synthetic_images(2, 320, seed=5).cuda(), **synthetic_labels(2, 80, seed=6)}
    tr.forward_backward(b)
    torch.cuda.synchronize()
    return tr.grad.clone(), tr


@pytest.mark.parametrize("cuts", [(13,), (19,), (20,), (7, 10, 20), None])
def test_staged_backward_matches_unstaged(cuts):
    from adrefine.engine.ddp import cuts_for_bucket
    ref, tr0 = _arena(())
    if cuts is None:
        cuts = cuts_for_bucket(tr0.model, 4.0)
    got, tr = _arena(cuts)
    # the arenas are laid out per stage: compare parameter by parameter
    g0 = {n: ref[tr0._goff[i]:tr0._goff[i] + t.numel()] for i, (n, t, _, isp) in enumerate(tr0.entries) if isp}
    g1 = {n: got[tr._goff[i]:tr._goff[i] + t.numel()] for i, (n, t, _, isp) in enumerate(tr.entries) if isp}
    assert set(g0) == set(g1)
    bad = []
    for n in g0:
        a, b = g0[n].double(), g1[n].double()
        if float((a - b).abs().max()) > 1e-4 * float(a.abs().max()) + 1e-7:
            bad.append((n, float((a - b).abs().max()), float(a.abs().max())))
    assert not bad, bad[:8]
