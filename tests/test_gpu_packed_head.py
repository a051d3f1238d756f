"""Level-packed AYHead (AYHead1._packed: the three pyramid levels in one row space, kernels.LevelPack) against the
reference's per-level loop (AYHead1._level, head.py:1132-1176). Same math, different summation order (GroupNorm /
pooling statistics over sub-images, the levels' WGRAD slabs reduced together), so the comparison is numeric:
fp32 to 1e-4 relative, bf16 to the bf16 engine's tolerance. Covers the head alone through plain autograd (fresh
gradient buffers, non-deferred parameter reductions) and the whole trainer (gradient arena, deferred reductions,
hipGraph replay), train and eval."""
import copy

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _nhwc(n, c, h, w, dtype, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(n, h, w, c, device="cuda", generator=g).to(dtype).permute(0, 3, 1, 2).detach()


@pytest.mark.parametrize("dtype,img,tol", [(torch.float32, 320, 1e-4), (torch.float32, 256, 1e-4),
                                           (torch.bfloat16, 320, 3e-2)])
def test_head_packed_matches_levels_autograd(dtype, img, tol):
    from adrefine import kernels as K
    from adrefine.nn.modules.head import AYHead1
    torch.manual_seed(0)
    ch = (64, 128, 256)
    ref = AYHead1(80, ch).cuda().train()
    ref.stride = torch.tensor([8.0, 16.0, 32.0])
    pk = copy.deepcopy(ref)
    ref.packed, pk.packed = False, True
    xs = [_nhwc(2, c, img // s, img // s, dtype, 10 + i) for i, (c, s) in enumerate(zip(ch, (8, 16, 32)))]
    gs = [_nhwc(2, 144, img // s, img // s, dtype, 20 + i) for i, s in enumerate((8, 16, 32))]
    res = []
    for m in (ref, pk):
        x = [t.clone().requires_grad_(True) for t in xs]
        K.relayout_count[0] = 0
        out = m(x)
        assert K.relayout_count[0] == 0
        loss = sum((o.float() * g.float()).sum() for o, g in zip(out, gs))
        loss.backward()
        torch.cuda.synchronize()
        res.append(([o.detach().clone() for o in out], [t.grad.clone() for t in x],
                    {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                    {n: b.clone() for n, b in m.named_buffers()}))
    (o0, dx0, g0, b0), (o1, dx1, g1, b1) = res
    for a, b in zip(o1, o0):
        assert a.shape == b.shape and _rel(a, b) < tol, _rel(a, b)
    for a, b in zip(dx1, dx0):
        assert _rel(a, b) < tol * (10 if dtype == torch.bfloat16 else 1), _rel(a, b)
    assert set(g0) == set(g1)
    # a bias feeding a training-mode BatchNorm (CoordAtt.conv1) has an exactly-zero gradient: both sides are
    # rounding noise, compared on the scale of the conv's weight gradient instead
    zero = {"coord_attention_reg.conv1.bias": ("coord_attention_reg.conv1.weight", 1e-3)}
    # TaskDecomposition's layer-attention gate scales each image's conv output right before a GroupNorm, which is
    # invariant to that scale: the gate's gradient (and la_conv1 / la_conv2's) is exactly zero in exact arithmetic,
    # rounding noise in both paths (bf16: noise of the bf16 activations) — bounded against the head's conv grads
    for d in ("cls_decomp", "reg_decomp"):
        for q in ("la_conv1.weight", "la_conv1.bias", "la_conv2.weight", "la_conv2.bias"):
            zero[f"{d}.{q}"] = (f"{d}.reduction_conv.conv.weight", 1e-3 if dtype == torch.float32 else 3e-2)
    for n, (w, f) in zero.items():
        scale = float(g0[w].norm())
        r0, r1 = float(g0.pop(n).norm()) / scale, float(g1.pop(n).norm()) / scale
        assert r0 < f and r1 < f, (n, r0, r1)
    bad = {n: _rel(g1[n], g0[n]) for n in g0 if _rel(g1[n], g0[n]) > tol * 10}
    assert not bad, bad
    for n in b0:  # CoordAtt's BatchNorm: per-level batch statistics, running stats updated level by level
        assert _rel(b1[n], b0[n]) < tol, (n, _rel(b1[n], b0[n]))


def _model(dtype):
    from adrefine.nn.tasks import DetectionModel
    from gpu_util import load_recipe_into
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


def _train(dtype, packed, graph, bs=4, img=320):
    from adrefine.data.synthetic import train_batch
    from adrefine.engine.trainer import FusedTrainer
    m = _model(dtype)
    m.model[-1].packed = packed
    tr = FusedTrainer(m, batch_size=bs, nbs=bs)
    b0, _ = train_batch(bs, img, seed=3, device="cuda", u8=True)
    b1, _ = train_batch(bs, img, seed=4, device="cuda", u8=True)
    tr.forward_backward(b0)
    torch.cuda.synchronize()
    arena0 = tr.grad.clone()
    items = [tr.step(b0)]
    if graph:
        tr.capture(b1)
    items.append(tr.step(b1))
    torch.cuda.synchronize()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    tr.graphs = None
    return torch.stack(items).float().cpu(), arena0, sd


@pytest.mark.parametrize("dtype,graph,tol", [(torch.float32, False, 1e-4), (torch.bfloat16, True, 5e-2)])
def test_trainer_packed_matches_levels(dtype, graph, tol):
    i0, a0, s0 = _train(dtype, False, graph)
    i1, a1, s1 = _train(dtype, True, graph)
    assert torch.isfinite(i1).all()
    assert _rel(i1, i0) < tol, (i0, i1)
    assert _rel(a1, a0) < tol, _rel(a1, a0)
    bad = {k: _rel(s1[k], s0[k]) for k in s0 if s0[k].is_floating_point() and s0[k].numel() > 1
           and _rel(s1[k], s0[k]) > tol}
    assert not bad, list(bad.items())[:10]


def test_eval_packed_matches_levels():
    from adrefine import kernels as K
    from adrefine.data.synthetic import images_u8
    m = _model(torch.float32).eval()
    x = images_u8(2, 320, seed=9).cuda()
    outs = []
    for packed in (False, True):
        m.model[-1].packed = packed
        with torch.no_grad(), K.pack_scope(K.PackCache(cache_bn_coefs=True)):
            y = m(x)
        torch.cuda.synchronize()
        outs.append(y[0].clone())
    assert _rel(outs[1], outs[0]) < 1e-4
