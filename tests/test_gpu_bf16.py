"""bf16 (the benchmarked compute dtype) at whole-network level against the reference, with stated bounds.

bf16 keeps 8 mantissa bits. On this network in TRAIN mode (batch-statistics BatchNorm, recipe weights) that
alone moves the head outputs by 17-33 % relative L2 away from fp32: measured with tests/bf16_sim.py, the
reference's own forward (the CPU oracle) with every functional op's output rounded to bf16, at 320^2 bs 2,
640^2 bs 4 and 320^2 bs 16 alike; eval mode (running statistics) moves only 1.5-2.7 %. The loss itself stays
within 0.3-2.5 %. So the bf16 bounds are stated against that ideal-bf16 restatement, computed in the test:

* train step, 701 yaml, 320^2 bs 2 vs the fp32 fixture net701_train_320: each head output's relative L2
  within 1.25x the ideal-bf16 divergence (+0.01); total loss and each of the three items within 3 %; the
  fraction of per-parameter gradient norms within 10 % of the fixture (floor 1e-3 of the largest) no more than
  0.05 below the ideal-bf16 restatement's own fraction;
* eval forward, 701 yaml, 640^2 bs 1 vs net701_eval_640: decoded boxes within 1 % relative L2 and 2 px max
  for anchors whose best class score exceeds 0.05, class scores within 0.03 absolute;
* full benchmark size (640^2, bs 64, bf16): a captured hipGraph step vs an eager step from the same state and
  batch, within 10x the eager-vs-eager run-to-run spread (DCN col2im's unordered float atomics)."""
import pytest
import torch

from bf16_sim import oracle_forward
from conftest import ROOT, golden, state_dict_spec
from gpu_util import load_recipe_into
from recipe import recipe_state_dict, synthetic_images

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _model(dtype):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


def _rel_l2(a, b):
    a, b = a.double().cpu(), torch.as_tensor(b).double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _gn_within(gn, ref, tol=0.10):
    """Fraction of parameters whose gradient norm is within tol (relative) of the fixture, with a floor of 1e-3
    of the largest norm (gradients that vanish in exact arithmetic — a conv bias feeding batch-statistics BN —
    are rounding noise in both)."""
    floor = 1e-3 * max(ref.values())
    rel = [(abs(gn.get(k, 0.0) - v) / (tol * v + floor), k) for k, v in ref.items()]
    return sum(r <= 1.0 for r, _ in rel) / len(rel), sorted(rel, reverse=True)[:3]


def test_bf16_train_step_vs_fixture():
    import adr_oracle as O
    g = golden("net701_train_320")
    x = synthetic_images(2, 320, seed=int(g["img_seed"]))
    lab = {k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}
    ref = dict(zip([str(k) for k in g["gn_keys"]], g["gn"]))
    # ideal-bf16 restatement on the CPU: its head-output divergence and gradient-norm agreement
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec("701")])
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k and not k.endswith("dfl.conv.weight"):
            v.requires_grad_(True)
    sp = oracle_forward(P, CFG, x, train=True, bf16=True)
    sloss, _ = O.detection_loss(sp, lab["batch_idx"], lab["cls"], lab["bboxes"])
    sloss.backward()
    sim_div = [_rel_l2(p.detach(), g[f"pred{i}"]) for i, p in enumerate(sp)]
    sim_within, _ = _gn_within({k: float(v.grad.norm()) for k, v in P.items() if v.grad is not None}, ref)
    # the HIP bf16 path
    m = _model(torch.bfloat16).train()
    preds = m.predict(x.cuda())
    div = [_rel_l2(p.float(), g[f"pred{i}"]) for i, p in enumerate(preds)]
    print(f"head rel L2: HIP bf16 {[round(d, 4) for d in div]}, ideal bf16 {[round(d, 4) for d in sim_div]}")
    for d, s in zip(div, sim_div):
        assert d <= 1.25 * s + 0.01, (div, sim_div)
    loss, items = m.loss({"img": x.cuda(), **lab}, preds=preds)
    dl = abs(float(loss) - float(g["loss"])) / float(g["loss"])
    di = ((items.float().cpu() - torch.from_numpy(g["items"]).float()).abs() /
          torch.from_numpy(g["items"]).float().abs()).max().item()
    print(f"loss rel {dl:.4f}, items max rel {di:.4f}")
    assert dl <= 0.03 and di <= 0.03, (dl, di)
    loss.backward()
    params = dict(m.named_parameters())
    within, worst = _gn_within({k: float(p.grad.norm()) for k, p in params.items() if p.grad is not None}, ref)
    print(f"grad norms within 10 %: HIP bf16 {within:.3f}, ideal bf16 {sim_within:.3f}; worst {worst}")
    assert within >= sim_within - 0.05, (within, sim_within, worst)


def test_bf16_eval_640_vs_fixture():
    g = golden("net701_eval_640")
    m = _model(torch.bfloat16).eval()
    x = synthetic_images(1, 640, seed=int(g["img_seed"])).cuda()
    with torch.no_grad():
        y, _ = m(x)
    ref = torch.as_tensor(g["y"]).float()
    y = y.float().cpu()
    rb = _rel_l2(y[:, :4], ref[:, :4])
    ds = float((y[:, 4:] - ref[:, 4:]).abs().max())
    conf = ref[:, 4:].amax(1) > 0.05  # (1, A) anchors that could survive a predict-time conf threshold
    dbox = float((y[:, :4] - ref[:, :4]).abs().amax(1)[conf].max()) if conf.any() else 0.0
    print(f"boxes rel L2 {rb:.4f}, max box err on scored anchors {dbox:.3f} px ({int(conf.sum())}), "
          f"max score err {ds:.4f}")
    assert rb <= 0.01 and ds <= 0.03 and dbox <= 2.0, (rb, ds, dbox)


def test_bf16_full_size_graph_step_matches_eager():
    """Two eager trainers give the run-to-run spread (DCN col2im accumulates with unordered float atomics);
    the captured step must stay within 10x that spread of the eager one (plus 1e-4 relative)."""
    from adrefine.data.synthetic import train_batch
    from adrefine.engine.trainer import FusedTrainer
    torch.manual_seed(0)
    batch, _ = train_batch(64, 640, seed=0, device="cuda")
    res = []
    for graph in (False, False, True):
        m = _model(torch.bfloat16)
        tr = FusedTrainer(m, batch_size=64)
        init = {k: v.detach().clone() for k, v in m.state_dict().items() if v.dtype.is_floating_point}
        tr.step(batch)  # step 1 eager in all (builds the tables and pack cache)
        if graph:
            tr.capture(batch)
        items = tr.step(batch).float().cpu()
        torch.cuda.synchronize()
        res.append((items, {k: v.detach().clone() for k, v in m.state_dict().items() if k in init}, init))
        del tr, m
    (ie, pe, init), (ie2, pe2, _), (ig, pg, _) = res
    assert torch.isfinite(ie).all() and torch.isfinite(ig).all()
    spread = float(((ie - ie2).abs() / ie.abs()).max())
    dgi = float(((ie - ig).abs() / ie.abs()).max())

    def upd(pa, pb):
        worst = 0.0
        for k in pa:
            if "running" in k or "num_batches" in k:
                continue
            delta = float((pa[k] - init[k]).norm())
            if delta == 0.0:
                continue
            worst = max(worst, float((pa[k] - pb[k]).norm()) / delta)
        return worst
    pspread, pd = upd(pe, pe2), upd(pe, pg)
    print(f"items: eager-eager {spread:.2e}, eager-graph {dgi:.2e}; updates: eager-eager {pspread:.3f}, "
          f"eager-graph {pd:.3f}")
    assert dgi <= 10 * spread + 1e-4, (ie, ie2, ig)
    assert pd <= 10 * pspread + 1e-3, (pd, pspread)
