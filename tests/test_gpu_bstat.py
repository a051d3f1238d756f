"""BN backward statistics in the consumer's data-gradient epilogue (BSTAT, adr_conv2d_dgrad_bf16_bstat).

A lazy BN-act output (Conv.forward(lazy=True): Bottleneck cv1 -> cv2, Conv layers feeding a Conv / C2f / SPPF) has one
reader, the conv that stages it, so that conv's data gradient is the BN's complete dz. The epilogue reads the BN
input y at the stored element and accumulates (sum g, sum g * y), g = dz * act'(y * s + t) — the terms adr_nc_reduce's
backward mode sums — and BNActFn.backward finalizes from those partials. Reference: Conv.forward =
act(bn(conv(x))) (nn/modules/conv.py:48-50) and BatchNorm2d's backward.

Checks: (1) per data-gradient path of the bf16 engine (streaming 1x1, implicit GEMM, stride-2 parity classes with
empty class tiles, 3x3 halo tiles, the wide 3x3 tile): dx is BITWISE the plain data gradient's, and the column sums
of the partials equal adr_nc_reduce's on the same (y, dx) to fp32 summation-order tolerance (1e-5 of sum |g|);
(2) a Conv -> Conv pair with the XF backward in the consumer's dgrad: the fused and unfused BN backward agree (the
sums are re-associated, so dx / dgamma / dbeta are compared at bf16-rounding tolerance, not bitwise) and the result
is deterministic; (3) the whole 701 bf16 train step: the same loss, BSTAT taken at >= 10 BatchNorms (that many fewer
nc_reduce launches), gradients within bf16 re-association noise of the unfused step."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _xf_everywhere(monkeypatch):
    """BSTAT with the XF operand transform on every kernel family, including the ones whose XF path the engine
    declines by default (adr_conv2d_bf16_xf_reuse)."""
    monkeypatch.setenv("ADR_XF_STREAM", "1")
    monkeypatch.setenv("ADR_XF_DG2", "1")
    monkeypatch.setenv("ADR_XF_CONV3", "1")


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


CASES = [  # n, C (dx channels = BN channels), K (dy channels), k, s, h, w, path
    (4, 64, 64, 1, 1, 20, 20, "conv1"),
    (2, 128, 192, 1, 1, 24, 24, "conv1 two column tiles"),
    (2, 320, 64, 1, 1, 10, 10, "implicit GEMM 1x1 (C > 256)"),
    (2, 64, 32, 3, 1, 13, 11, "implicit GEMM 3x3 (odd width)"),
    (2, 16, 32, 3, 2, 40, 40, "stride-2 parity classes"),
    (2, 64, 128, 3, 2, 21, 19, "stride-2, odd sizes"),
    (1, 32, 32, 3, 2, 23, 23, "stride-2: a parity class with a tile past its rows (zero statistics row)"),
    (4, 64, 64, 3, 1, 16, 16, "3x3 halo tiles TW 16"),
    (2, 32, 64, 3, 1, 24, 8, "3x3 halo tiles TW 8"),
    (16, 256, 128, 3, 1, 64, 64, "3x3 wide tile"),
]


@pytest.mark.parametrize("act", ["silu", "none"])
@pytest.mark.parametrize("n,C,Kc,k,s,h,w,path", CASES)
def test_dgrad_bstat_kernel(n, C, Kc, k, s, h, w, path, act):
    from adrefine import kernels as K
    from adrefine.native import lib
    torch.manual_seed(0)
    dev = "cuda"
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    dy = _nhwc(torch.randn(n, Kc, ho, wo, device=dev).to(torch.bfloat16))
    wt = torch.randn(Kc, C, k, k, device=dev) * (1.0 / (C * k * k) ** 0.5)
    y = _nhwc((torch.randn(n, C, h, w, device=dev) * 2).to(torch.bfloat16))
    scale = torch.rand(C, device=dev) + 0.5
    shift = torch.randn(C, device=dev) * 0.3
    _, crsk = K.pack_weight2(wt, torch.bfloat16)
    d, _, _ = K.conv_desc(n, h, w, C, C, Kc, k, k, s, s, p, p, Kc, torch.bfloat16)
    dx0 = K.empty_act(n, C, h, w, torch.bfloat16, dev)
    lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(crsk.data_ptr()),
                              None, ctypes.c_void_p(dx0.data_ptr()), 0, K.stream())
    P = lib.adr_conv2d_dgrad_bf16_stat_tiles(ctypes.byref(d), 0)
    part = torch.full((P * 2 * C,), float("nan"), device=dev)
    dx1 = K.empty_act(n, C, h, w, torch.bfloat16, dev)
    bs = K.BStatStruct(y.data_ptr(), scale.data_ptr(), shift.data_ptr(), C, K.ACT[act])
    lib.adr_conv2d_dgrad_bf16_bstat(ctypes.byref(d), ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(crsk.data_ptr()),
                                    ctypes.c_void_p(dx1.data_ptr()), 0, None, 0, None, ctypes.byref(bs),
                                    K.fptr(part), K.stream())
    assert torch.equal(dx0, dx1), path  # the data gradient itself is the plain kernel's
    assert bool(torch.isfinite(part).all()), f"{path}: unwritten statistics rows"
    got = part.view(P, 2, C).double().sum(0)
    # adr_nc_reduce's backward partials on the same (y, dz) as the reference of the per-element terms
    HW = h * w
    rows = K._stats_rows(n, HW)
    chunks = lib.adr_nc_reduce_chunks(HW, rows)
    ref = torch.empty(n * chunks * 2 * C, device=dev)
    lib.adr_nc_reduce(K.dcode(torch.bfloat16), 1, ctypes.c_void_p(y.data_ptr()), C, 0,
                      ctypes.c_void_p(dx0.data_ptr()), C, 0, K.fptr(scale), K.fptr(shift), 0, K.ACT[act], n, HW, C,
                      rows, K.fptr(ref), K.stream())
    want = ref.view(-1, 2, C).double().sum(0)
    # scale of the sums: sum |g| and sum |g * y| in float64 from the same operands
    yf, dzf = y.double(), dx0.double()
    v = yf * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)
    sg = torch.sigmoid(v)
    g = dzf * (sg * (1 + v * (1 - sg)) if act == "silu" else 1.0)
    mag = torch.stack((g.abs().sum((0, 2, 3)), (g * yf).abs().sum((0, 2, 3))))
    err = float(((got - want).abs() / (mag + 1e-30)).max())
    assert err < 1e-5, (path, err)


def _pair(c1, c, k1, s1, k2):
    from adrefine.nn.modules.conv import Conv
    p = Conv(c1, c, k1, s1).cuda().train()
    q = Conv(c, c, k2, 1).cuda().train()
    with torch.no_grad():
        for m in (p, q):
            m.bn.weight.uniform_(0.5, 1.5)
            m.bn.bias.uniform_(-0.3, 0.3)
    return p, q


def _pair_run(p, q, x, g, bstat):
    from adrefine import kernels as K
    old = K.BN_BSTAT
    K.BN_BSTAT = bstat
    sd = ({k: v.clone() for k, v in p.state_dict().items()}, {k: v.clone() for k, v in q.state_dict().items()})
    try:
        xx = x.detach().clone().requires_grad_(True)
        z2 = q(p(xx, lazy=True))
        z2.backward(g)
        torch.cuda.synchronize()
        res = [z2.detach().clone(), xx.grad.clone()]
        res += [t.grad.clone() for t in (p.conv.weight, p.bn.weight, p.bn.bias, q.conv.weight, q.bn.weight, q.bn.bias)]
    finally:
        K.BN_BSTAT = old
        p.zero_grad(set_to_none=True)
        q.zero_grad(set_to_none=True)
        p.load_state_dict(sd[0])
        q.load_state_dict(sd[1])
    return res


PAIRS = [  # n, c1, c, k1, s1, k2, h, w
    (4, 32, 32, 3, 1, 3, 16, 16),   # bottleneck 3x3 -> 3x3 (halo tiles; the consumer's dgrad with XF backward)
    (4, 16, 32, 3, 2, 1, 40, 40),   # Conv s2 -> 1x1 (the consumer's 1x1 dgrad)
    (2, 64, 128, 3, 2, 1, 20, 20),  # 1x1 128 -> 128
]


@pytest.mark.parametrize("n,c1,c,k1,s1,k2,h,w", PAIRS)
def test_pair_bstat_matches_nc_reduce(n, c1, c, k1, s1, k2, h, w):
    torch.manual_seed(1)
    p, q = _pair(c1, c, k1, s1, k2)
    x = _nhwc((torch.randn(n, c1, h, w, device="cuda") * 1.5).to(torch.bfloat16))
    ho, wo = (h + 2 * (k1 // 2) - k1) // s1 + 1, (w + 2 * (k1 // 2) - k1) // s1 + 1
    g = _nhwc(torch.randn(n, c, ho, wo, device="cuda").to(torch.bfloat16))
    a = _pair_run(p, q, x, g, True)
    a2 = _pair_run(p, q, x, g, True)
    b = _pair_run(p, q, x, g, False)
    names = ("out", "dx", "dw1", "dgamma1", "dbeta1", "dw2", "dgamma2", "dbeta2")
    for name, u, v in zip(names, a, a2):
        assert torch.equal(u, v), ("not deterministic", name)
    for name, u, v in zip(names, a, b):
        if name in ("out", "dw2", "dgamma2", "dbeta2"):  # the consumer's own BN backward is unchanged
            assert torch.equal(u, v), name
            continue
        rel = float((u.double() - v.double()).norm() / (v.double().norm() + 1e-30))
        assert rel < 5e-3, (name, rel)  # re-associated fp32 sums -> a few 1-ulp bf16 flips of dy downstream


def test_whole_net_step_bstat():
    """One bf16 train step of the 701 graph at 320^2 bs 2 with and without BSTAT: identical loss (the forward is
    untouched), BSTAT taken at >= 10 BatchNorms (14 measured) with that many fewer nc_reduce launches, and the change
    of the parameter gradients small against bf16's own error: |g_bstat - g_unfused| over all parameters <= 0.1 x
    |g_unfused - g_fp32| (the fp32 parity-mode step; measured 0.030), and <= 0.2 x for 90 % of the parameters
    (measured p95 0.096). Per parameter the ratio can reach ~1.4 only where the exact gradient is zero and both sides
    are rounding noise (conv biases in front of a normalisation, C2PTSSA's fusion stages)."""
    from adrefine import kernels as K
    from adrefine import native as NV
    from adrefine.nn.tasks import DetectionModel
    from conftest import ROOT
    from gpu_util import load_recipe_into
    from recipe import synthetic_images
    m = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16)
    load_recipe_into(m)
    m = m.cuda().train()
    img = synthetic_images(2, 320, seed=3).cuda()
    batch = {"img": img, "batch_idx": torch.tensor([0., 0., 1.]), "cls": torch.tensor([[1.], [5.], [7.]]),
             "bboxes": torch.tensor([[0.5, 0.5, 0.3, 0.4], [0.2, 0.3, 0.1, 0.2], [0.6, 0.6, 0.5, 0.3]])}
    runs = []
    for on in (True, False):
        old = K.BN_BSTAT
        K.BN_BSTAT = on
        counts = {}

        def hook(name, fn, args):
            key = name if name != "adr_nc_reduce" else f"{name}/{args[1]}"
            counts[key] = counts.get(key, 0) + 1
            rc = fn(*args)
            if rc != 0:
                raise RuntimeError(name)
            return rc
        NV.CALL_HOOK = hook
        try:
            sd = {k: v.clone() for k, v in m.state_dict().items()}
            loss, _ = m(batch)
            loss.backward()
            torch.cuda.synchronize()
            runs.append((float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                         counts))
            m.zero_grad(set_to_none=True)
            m.load_state_dict(sd)
        finally:
            NV.CALL_HOOK = None
            K.BN_BSTAT = old
    (la, ga, ca), (lb, gb, cb) = runs
    assert la == lb
    nb = ca.get("adr_conv2d_dgrad_bf16_bstat", 0)
    print(f"BSTAT launches {nb}; nc_reduce backward launches {ca.get('adr_nc_reduce/1', 0)} vs "
          f"{cb.get('adr_nc_reduce/1', 0)}")
    assert nb >= 10
    assert cb.get("adr_nc_reduce/1", 0) - ca.get("adr_nc_reduce/1", 0) == nb
    # the yardstick: bf16's own error, the same step in the fp32 parity mode (the reference-pinned path)
    m32 = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"))
    load_recipe_into(m32)
    m32 = m32.cuda().train()
    loss32, _ = m32(batch)
    loss32.backward()
    g32 = {n: p.grad.clone() for n, p in m32.named_parameters() if p.grad is not None}
    ratios, db_all, dp_all = [], 0.0, 0.0
    for n in ga:
        db = float((ga[n].double() - gb[n].double()).norm())
        dp = float((gb[n].double() - g32[n].double()).norm())
        db_all += db * db
        dp_all += dp * dp
        ratios.append((db / (dp + 1e-30), n))
    ratios.sort()
    agg = (db_all / dp_all) ** 0.5
    print(f"|bstat - unfused| / |unfused - fp32|: aggregate {agg:.3e}, median {ratios[len(ratios) // 2][0]:.3e}, "
          f"p95 {ratios[int(0.95 * len(ratios))][0]:.3e}, worst {ratios[-3:]}")
    assert agg <= 0.1, agg  # measured 0.030
    assert ratios[int(0.9 * len(ratios))][0] <= 0.2, ratios[int(0.9 * len(ratios)):]  # measured p95 0.096
