"""hipGraph capture of the training step (FusedTrainer.capture) reproduces eager steps: same loss items and
parameters after several steps, including a batch change (copied into the captured static inputs). The bar is
the run-to-run spread of two eager trainers (fp32 scatter atomics in the DCN backward are unordered)."""
import pytest
import torch

from conftest import ROOT
from gpu_util import load_recipe_into
from recipe import synthetic_images, synthetic_labels

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _trainer(stages=None):
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    return FusedTrainer(m.cuda(), nbs=2, batch_size=2, stages=stages)


def _run(seq, graph, stages=None):
    tr = _trainer(stages)
    out = [tr.step(seq[0]).clone()]
    if graph:
        tr.capture(seq[1], max_targets=100)
    out += [tr.step(b).clone() for b in seq[1:]]
    torch.cuda.synchronize()
    return tr, out


def _pdiff(a, b):
    sa, sb = a.model.state_dict(), b.model.state_dict()
    return max(float((sa[k] - sb[k]).abs().max()) for k in sa if sa[k].dtype.is_floating_point)


def test_graph_step_matches_eager():
    b1 = {"img": synthetic_images(2, 320, seed=0).cuda(), **synthetic_labels(2, 80, seed=1)}
    b2 = {"img": synthetic_images(2, 320, seed=5).cuda(), **synthetic_labels(2, 80, seed=6)}
    seq = [b1, b1, b2, b1]
    e1, o1 = _run(seq, False)
    e2, o2 = _run(seq, False)
    g, og = _run(seq, True)
    for a, b, c in zip(o1, og, o2):
        item_spread = float((a - c).abs().max())
        assert float((a - b).abs().max()) <= 10 * item_spread + 2e-4 * float(a.abs().max()), (a, b, c)
    spread = _pdiff(e1, e2)
    d = _pdiff(e1, g)
    print(f"eager-eager max |dparam| {spread:.3e}, eager-graph {d:.3e}")
    assert d <= 10 * spread + 2e-4, (d, spread)
    ee, eg = e1.ema_state_dict(), g.ema_state_dict()
    assert max(float((ee[k] - eg[k]).abs().max()) for k in ee) <= 10 * spread + 2e-4


@pytest.mark.parametrize("graph", [False, True])
def test_staged_step_matches_unstaged(graph):
    """The DDP stage split (backward in three stages L0-L6 | L7-L10 | L11-L33, one graph per stage when
    captured, engine/ddp.py) reproduces the single-stage step."""
    b1 = {"img": synthetic_images(2, 320, seed=0).cuda(), **synthetic_labels(2, 80, seed=1)}
    b2 = {"img": synthetic_images(2, 320, seed=5).cuda(), **synthetic_labels(2, 80, seed=6)}
    seq = [b1, b1, b2]
    e1, o1 = _run(seq, False)
    e2, o2 = _run(seq, False)
    st, os_ = _run(seq, graph, stages=(6, 10))
    assert st.cuts == (6, 10) and len(st.buckets) == 3
    if graph:
        assert len(st.graphs[0]) == 3
    spread = _pdiff(e1, e2)
    d = _pdiff(e1, st)
    print(f"eager-eager max |dparam| {spread:.3e}, unstaged-staged {d:.3e}")
    assert d <= 10 * spread + 2e-4, (d, spread)
    for a, b, c in zip(o1, os_, o2):
        assert float((a - b).abs().max()) <= 10 * float((a - c).abs().max()) + 2e-4 * float(a.abs().max())


def test_pack_cache_matches_direct_packing():
    """The trainer's batched once-per-step weight packing (PackCache.pack_all) produces exactly the operands a
    per-call adr_pack_weight2 would, for every recorded conv weight, after an optimizer update."""
    from adrefine import kernels as K
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG), compute_dtype=torch.bfloat16)
    load_recipe_into(m)
    tr = FusedTrainer(m.cuda(), nbs=2, batch_size=2)
    b = {"img": synthetic_images(2, 320, seed=0).cuda(), **synthetic_labels(2, 80, seed=1)}
    tr.step(b)
    tr.step(b)  # second step runs on pack_all's buffers; the weights have moved since
    assert len(tr.packs.specs) > 50
    tr.packs.pack_all()
    torch.cuda.synchronize()
    for (wid, cpad, tkc, kpad), sp in tr.packs.specs.items():
        w = sp[0]
        kr, cr = K.pack_weight2(w, torch.bfloat16, cpad, tkc, kpad)  # no active cache here: direct pack
        assert torch.equal(kr, sp[7]) and torch.equal(cr, sp[8]), tuple(w.shape)


def _labels_n(bs, n, seed):
    """Exactly n boxes per image (normalised xywh, classes 0..79): the per-image target count the captured step's
    static gt must hold."""
    g = torch.Generator().manual_seed(seed)
    ctr = 0.1 + 0.8 * torch.rand(bs * n, 2, generator=g)
    wh = 0.02 + 0.2 * torch.rand(bs * n, 2, generator=g)
    return {"batch_idx": torch.arange(bs).repeat_interleave(n).float(),
            "cls": torch.randint(0, 80, (bs * n, 1), generator=g).float(),
            "bboxes": torch.cat((ctr, wh), 1)}


def test_graph_step_grows_target_capacity():
    """A captured trainer fed batches with 7, then 93, then 7 and 93 targets per image (COCO's Poisson(7.3) counts
    reach ~93): no error mid-training — the 93-target batch captures a 128-capacity step (capacity_bucket) and later
    the smaller capture is dropped (graph memory stays one captured step) — and every step matches the eager trainer (fp32: loss items 1e-4
    relative, parameters and EMA within the eager-eager spread bound). Reference: utils/loss.py:392-408 pads the
    targets per batch; trainer.py:367-398 the step loop."""
    from adrefine.engine.trainer import FusedTrainer
    b7 = {"img": synthetic_images(2, 320, seed=0).cuda(), **_labels_n(2, 7, seed=1)}
    b93 = {"img": synthetic_images(2, 320, seed=5).cuda(), **_labels_n(2, 93, seed=6)}
    seq = [b7, b7, b93, b7, b93]

    def run(graph):
        tr = _trainer()
        out = [tr.step(seq[0]).clone()]
        if graph:
            tr.capture(seq[1])  # capacity 7, from the batch
            assert tr.static_batch["gt"].shape[1] == 7
        caps = []
        for b in seq[1:]:
            out.append(tr.step(b).clone())
            if graph:
                caps.append(tr.static_batch["gt"].shape[1])
        torch.cuda.synchronize()
        return tr, out, caps

    e1, o1, _ = run(False)
    e2, o2, _ = run(False)
    g, og, caps = run(True)
    assert caps == [7, 128, 128, 128] and FusedTrainer.capacity_bucket(93) == 128
    assert sorted(g._sets) == [128]
    for a, b, c in zip(o1, og, o2):
        spread = float((a - c).abs().max())
        assert float((a - b).abs().max()) <= 10 * spread + 1e-4 * float(a.abs().max()), (a, b, c)
    spread = _pdiff(e1, e2)
    d = _pdiff(e1, g)
    print(f"eager-eager max |dparam| {spread:.3e}, eager-graph {d:.3e}")
    assert d <= 10 * spread + 1e-4, (d, spread)
    ee, eg = e1.ema_state_dict(), g.ema_state_dict()
    assert max(float((ee[k] - eg[k]).abs().max()) for k in ee) <= 10 * spread + 1e-4


def test_graph_capacity_buckets_bounded_memory():
    """Walking through target-capacity buckets 8 -> 16 -> 32 -> 64 -> 128 keeps ONE captured step alive (ADVICE r05:
    each set owns a private pool holding a whole step's activations): the reserved memory after the last capture
    stays within 1.5x of what the first capture reserved."""
    tr = _trainer()
    bs = [{"img": synthetic_images(2, 320, seed=0).cuda(), **_labels_n(2, n, seed=1)} for n in (5, 12, 30, 60, 120)]
    tr.step(bs[0])
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_reserved()
    tr.capture(bs[0])
    torch.cuda.synchronize()
    one = torch.cuda.memory_reserved() - base
    for b in bs[1:]:
        tr.step(b)
    torch.cuda.synchronize()
    assert sorted(tr._sets) == [128]
    grown = torch.cuda.memory_reserved() - base
    print(f"one captured set {one / 2**20:.1f} MiB, after 4 bucket captures {grown / 2**20:.1f} MiB")
    assert grown <= 1.5 * one + (64 << 20), (one, grown)
