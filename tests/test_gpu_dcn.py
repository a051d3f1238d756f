"""DyDCNv2's modulated deformable conv (mmcv ModulatedDeformConv2d as head.py:751-782 calls it) on its own,
against the oracle's mmcv restatement (oracle/adr_oracle.py dcn_v2; mmcv itself is absent, so the
third-party core is 'parity unpinned' — the whole-head fixtures pin the reference's arithmetic around it).

Offsets spread to +-6 px, so samples leave the image and bilinear corners come from sources outside the bf16
backward's per-tap 12x12 source sub-window (the far-list path) as well as inside it; maps that are and are not
multiples of the 8x8 backward tile; C = Cout in {64, 128, 256} (the n- and l-scale AYHead widths) on the fused
backward, other shapes on the im2col path.

fp32 (parity mode, im2col + GEMM + deterministic col2im): outputs and all gradients within 1e-4 relative of
the fp64 oracle, and the input gradient is bitwise identical across two runs.
bf16 (fused kernels, adr_dcn.hip): against the oracle evaluated in fp64 on the bf16-rounded inputs, relative L2
within 1 % (y), 1.5 % (dx, dw) and 3 % (offset / mask-logit gradients, which sum products of bf16 values)."""
import pytest
import torch

import adr_oracle as O

pytestmark = pytest.mark.gpu

CASES = [  # (N, C, Cout, H, W, offset spread px)
    (4, 64, 64, 80, 80, 6.0),
    (2, 64, 64, 20, 20, 1.5),
    (3, 128, 64, 13, 11, 3.0),
    (2, 64, 128, 16, 24, 2.5),
    (2, 128, 128, 24, 20, 2.5),
    (2, 256, 256, 12, 16, 1.0),
    (1, 256, 256, 40, 40, 4.0),
]


def _inputs(N, C, Cout, H, W, spread, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g)
    om = torch.zeros(N, 32, H, W)
    om[:, :18] = (torch.rand(N, 18, H, W, generator=g) * 2 - 1) * spread
    om[:, 18:27] = torch.randn(N, 9, H, W, generator=g) * 2
    w = torch.randn(Cout, C, 3, 3, generator=g) * (9 * C) ** -0.5
    gy = torch.randn(N, Cout, H, W, generator=g)
    return x, om, w, gy


def _oracle(x, om, w, gy):
    x = x.double().requires_grad_(True)
    om = om.double().requires_grad_(True)
    w = w.double().requires_grad_(True)
    y = O.dcn_v2(x, om[:, :18], torch.sigmoid(om[:, 18:27]), w)
    y.backward(gy.double())
    return y.detach(), x.grad, om.grad, w.grad


def _run(x, om, w, gy, dtype):
    from adrefine import kernels as K
    dev = "cuda"
    xd = x.to(dev, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    omd = om.to(dev, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(dev).requires_grad_(True)
    y = K.dcn(xd, omd, wd)
    y.backward(gy.to(dev, dtype).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    return y.detach().double().cpu(), xd.grad.double().cpu(), omd.grad.double().cpu(), wd.grad.double().cpu()


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("case", CASES)
def test_dcn_fp32_vs_oracle_and_deterministic(case):
    N, C, Cout, H, W, spread = case
    x, om, w, gy = _inputs(N, C, Cout, H, W, spread, seed=7)
    ry, rdx, rdom, rdw = _oracle(x, om, w, gy)
    y, dx, dom, dw = _run(x, om, w, gy, torch.float32)
    # a sample coordinate within 1e-5 px of an integer may take the other bilinear cell in fp32 than in the fp64
    # oracle (e.g. offset 0.9999995 -> 18.0): the offset / mask gradients of that (pixel, tap) are discontinuous
    # there, so those entries are left out of the comparison
    fr = om[:, :18].double().frac().abs()
    edge = (torch.minimum(fr, 1 - fr) < 1e-5).view(N, 9, 2, H, W).any(2)
    keep = torch.ones(N, 32, H, W, dtype=torch.bool)
    keep[:, :18] = ~edge.repeat_interleave(2, 1)
    keep[:, 18:27] = ~edge
    dom, rdom = dom * keep, rdom * keep
    for name, a, b in (("y", y, ry), ("dx", dx, rdx), ("doffset", dom[:, :18], rdom[:, :18]),
                       ("dmask", dom[:, 18:27], rdom[:, 18:27]), ("dw", dw, rdw)):
        err = float((a - b).abs().max()) / float(b.abs().max())
        assert err <= 1e-4, (name, err)
    assert float(dom[:, 27:].abs().max()) == 0.0
    _, dx2, dom2, _ = _run(x, om, w, gy, torch.float32)
    dom2 = dom2 * keep
    assert torch.equal(dx, dx2) and torch.equal(dom, dom2), "fp32 parity-mode DCN backward is not repeatable"


@pytest.mark.parametrize("case", CASES)
def test_dcn_bf16_fused_vs_oracle(case):
    N, C, Cout, H, W, spread = case
    x, om, w, gy = _inputs(N, C, Cout, H, W, spread, seed=11)
    rnd = lambda t: t.bfloat16().float()  # noqa: E731 - the kernels see bf16 activations (weights stay fp32)
    ry, rdx, rdom, rdw = _oracle(rnd(x), rnd(om), rnd(w), rnd(gy))
    y, dx, dom, dw = _run(x, om, w, gy, torch.bfloat16)
    errs = {"y": _rel(y, ry), "dx": _rel(dx, rdx), "doffset": _rel(dom[:, :18], rdom[:, :18]),
            "dmask": _rel(dom[:, 18:27], rdom[:, 18:27]), "dw": _rel(dw, rdw)}
    print(case, {k: round(v, 5) for k, v in errs.items()})
    bounds = {"y": 0.01, "dx": 0.015, "doffset": 0.03, "dmask": 0.03, "dw": 0.015}
    for k, v in errs.items():
        assert v <= bounds[k], (k, v, errs)
    assert float(dom[:, 27:].abs().max()) == 0.0


@pytest.mark.parametrize("C", [64, 128, 256])
def test_dcn_bf16_backward_repeatable_near(C):
    """|offsets| < 2 px: every corner is gathered by its destination tile (no far entries), so the bf16 backward
    is bitwise repeatable."""
    x, om, w, gy = _inputs(2, C, C, 24, 17, 1.9, seed=5)
    _, dx, dom, dw = _run(x, om, w, gy, torch.bfloat16)
    _, dx2, dom2, dw2 = _run(x, om, w, gy, torch.bfloat16)
    assert torch.equal(dx, dx2) and torch.equal(dom, dom2) and torch.equal(dw, dw2)


@pytest.mark.parametrize("C", [64, 128])
def test_dcn_levels_one_launch_bitwise(C):
    """The AYHead's three pyramid levels in one launch per direction (adr_dcn_{fwd,bwd,wgrad}_bf16_levels, the
    level-packed head's LevelDCNFn) against one launch per level: output, input / offset / weight gradients
    bitwise equal (|offsets| < 2 px, so the backward has no far-corner atomics)."""
    from adrefine import kernels as K
    N, dims = 2, [(24, 24), (12, 12), (6, 6)]
    pack = K.LevelPack(N, dims)
    g = torch.Generator().manual_seed(9)
    xs = [torch.randn(N, C, H, W, generator=g) for H, W in dims]
    oms = []
    for H, W in dims:
        om = torch.zeros(N, 32, H, W)
        om[:, :18] = (torch.rand(N, 18, H, W, generator=g) * 2 - 1) * 1.8
        om[:, 18:27] = torch.randn(N, 9, H, W, generator=g) * 2
        oms.append(om)
    w = torch.randn(C, C, 3, 3, generator=g) * (9 * C) ** -0.5
    gys = [torch.randn(N, C, H, W, generator=g) for H, W in dims]
    runs = []
    for levels in (True, False):
        old = K.DCN_LEVELS
        K.DCN_LEVELS = levels
        try:
            xd = [t.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True) for t in xs]
            od = [t.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True) for t in oms]
            wd = w.cuda().requires_grad_(True)
            y = K.dcn_levels(K.level_join(xd, pack), K.level_join(od, pack), wd, pack)
            ys = K.level_split(y, pack)
            torch.autograd.backward(list(ys), [t.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                                               for t in gys])
            torch.cuda.synchronize()
            runs.append([y.detach().clone()] + [t.grad.clone() for t in xd] + [t.grad.clone() for t in od] +
                        [wd.grad.clone()])
        finally:
            K.DCN_LEVELS = old
    for i, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), i


def test_dcn_levels_far_scratch_reused():
    """Two eager LevelDCNFn backwards of the same shape reuse ONE persistent far-corner scratch pair: no new
    allocation, nothing retired (the prefix-view size check reallocated it on every call)."""
    from adrefine import kernels as K
    N, C, dims = 2, 64, [(24, 24), (12, 12), (6, 6)]
    pack = K.LevelPack(N, dims)
    g = torch.Generator().manual_seed(3)
    old = K.DCN_LEVELS
    K.DCN_LEVELS = True
    try:
        ptrs = []
        for rep in range(3):
            xd = [torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16)
                  .contiguous(memory_format=torch.channels_last).requires_grad_(True) for H, W in dims]
            od = [(torch.randn(N, 32, H, W, generator=g) * 3).cuda().to(torch.bfloat16)
                  .contiguous(memory_format=torch.channels_last).requires_grad_(True) for H, W in dims]
            wd = (torch.randn(C, C, 3, 3, generator=g) * (9 * C) ** -0.5).cuda().requires_grad_(True)
            y = K.dcn_levels(K.level_join(xd, pack), K.level_join(od, pack), wd, pack)
            y.float().square().sum().backward()
            torch.cuda.synchronize()
            f, fl = K._DCN_FAR[str(xd[0].device)]
            ptrs.append((f.data_ptr(), fl.data_ptr(), len(K._DCN_FAR_RETIRED)))
        assert ptrs[1] == ptrs[2], ptrs
        # the kernels leave the scratch zero again
        assert float(K._DCN_FAR[str(xd[0].device)][0].abs().max()) == 0.0
    finally:
        K.DCN_LEVELS = old
