"""GPU parity: dense conv family (Conv-BN-SiLU, nn.Conv2d+bias, ConvTranspose2d) vs the CPU oracle."""
import pytest
import torch

import adr_oracle as O
from conftest import golden
from gpu_util import TOL, assert_close, load_recipe_into, param_dict_requires_grad, to_dev
from recipe import recipe_state_dict, seeded_randn

pytestmark = pytest.mark.gpu


def _prefixed(P, pre="m"):
    return {pre + "." + k: v for k, v in P.items()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c1,c2,k,s,hw", [(16, 32, 3, 2, 24), (32, 64, 1, 1, 20), (64, 128, 3, 1, 13),
                                           (128, 256, 3, 2, 20), (48, 16, 1, 1, 9), (8, 16, 3, 1, 7),
                                           (32, 32, 3, 2, 15), (16, 16, 1, 2, 9),
                                           # 3x3 halo-tile path (adr_conv.hip conv3_kernel): 16- and 8-wide tiles,
                                           # ragged last tile row band, one and several 32-channel chunks
                                           (64, 64, 3, 1, 16), (64, 128, 3, 1, 24), (32, 64, 3, 1, 40),
                                           (128, 64, 3, 1, 16), (64, 32, 3, 1, 16), (32, 32, 3, 1, 24),
                                           # thin-channel 3x3 halo WGRAD (adr_wgrad.hip wgrad3t_kernel): C <= 16,
                                           # K <= 32, stride 1 and 2, padded channel blocks
                                           (16, 8, 3, 1, 32), (8, 16, 3, 1, 32), (16, 32, 3, 2, 64),
                                           (8, 32, 3, 2, 32)])
def test_conv_bn_silu(dtype, c1, c2, k, s, hw):
    from adrefine.nn.modules import Conv
    m = Conv(c1, c2, k, s)
    rec = load_recipe_into(m)
    m = m.cuda().train()
    x = seeded_randn(2, c1, hw, hw, seed=5)
    xd = to_dev(x, dtype)
    y = m(xd)
    g = seeded_randn(*y.shape, seed=6)
    y.backward(g.to("cuda", dtype))
    P = param_dict_requires_grad({k2: v.clone() for k2, v in rec.items()})
    xr = x.clone().requires_grad_(True)
    yr = O.conv_bn_act(_prefixed(P), "m", xr, k, s)
    yr.backward(g)
    tol = TOL[dtype]
    assert_close(y.float(), yr, **tol, what="y")
    assert_close(xd.grad.float(), xr.grad, **tol, what="dx")
    assert_close(m.conv.weight.grad, P["conv.weight"].grad, **tol, what="dw")
    assert_close(m.bn.weight.grad, P["bn.weight"].grad, **tol, what="dgamma")
    assert_close(m.bn.bias.grad, P["bn.bias"].grad, **tol, what="dbeta")
    assert_close(m.bn.running_mean, P["bn.running_mean"], rtol=1e-4, atol=1e-4 if dtype == torch.float32 else 2e-2,
                 what="running_mean")
    assert_close(m.bn.running_var, P["bn.running_var"], rtol=1e-4, atol=1e-4 if dtype == torch.float32 else 2e-2,
                 what="running_var")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_c3k2_bottleneck_thin_sliced(dtype):
    """The C3k2 bottleneck of model.2 at a tile-aligned size: its 16 -> 8 3x3 conv reads a 16-channel slice of the
    48-channel concat buffer (x channel stride 48) and runs the thin-channel WGRAD kernel."""
    from adrefine.nn.modules.block import C3k2
    m = C3k2(32, 64, 1, False, 0.25)
    rec = load_recipe_into(m)
    m = m.cuda().train()
    x = seeded_randn(2, 32, 32, 32, seed=7)
    xd = to_dev(x, dtype)
    y = m(xd)
    g = seeded_randn(*y.shape, seed=8)
    y.backward(g.to("cuda", dtype))
    P = param_dict_requires_grad({k2: v.clone() for k2, v in rec.items()})
    xr = x.clone().requires_grad_(True)
    yr = O.c2f_family(_prefixed(P), "m", xr, 32, 64, 1, False, 0.25, True, True, False)
    yr.backward(g)
    tol = TOL[dtype]
    assert_close(y.float(), yr, **tol, what="y")
    assert_close(xd.grad.float(), xr.grad, **tol, what="dx")
    for name, prm in m.named_parameters():
        assert_close(prm.grad, P[name].grad, **tol, what=name)


def test_conv_golden_fixture():
    """Same module against the reference-generated fixture directly (fp32)."""
    from adrefine.nn.modules import Conv
    g = golden("mod_conv_k3s2")
    m = Conv(16, 32, 3, 2)
    load_recipe_into(m)
    m = m.cuda().train()
    x = seeded_randn(*[int(v) for v in g["in0_shape"]], seed=int(g["in0_seed"]))
    xd = to_dev(x, torch.float32)
    y = m(xd)
    gen = torch.Generator().manual_seed(22)
    gout = torch.randn(y.shape, generator=gen)
    y.backward(gout.cuda())
    assert_close(y, g["out0"], rtol=1e-4, atol=1e-4, what="y")
    assert_close(xd.grad, g["gin0"], rtol=1e-4, atol=1e-4, what="dx")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv2d_bias(dtype):
    from adrefine.nn.modules import Conv2d
    m = Conv2d(256, 128, 1)
    rec = load_recipe_into(m)
    m = m.cuda()
    x = seeded_randn(2, 256, 10, 10, seed=8)
    xd = to_dev(x, dtype)
    y = m(xd)
    gy = seeded_randn(*y.shape, seed=9)
    y.backward(gy.to("cuda", dtype))
    P = param_dict_requires_grad({k: v.clone() for k, v in rec.items()})
    xr = x.clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, P["weight"], P["bias"])
    yr.backward(gy)
    tol = TOL[dtype]
    assert_close(y.float(), yr, **tol, what="y")
    assert_close(xd.grad.float(), xr.grad, **tol, what="dx")
    assert_close(m.weight.grad, P["weight"].grad, **tol, what="dw")
    assert_close(m.bias.grad, P["bias"].grad, **tol, what="db")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_transpose_fixture(dtype):
    from adrefine.nn.modules import ConvTranspose2d
    g = golden("mod_convT")
    m = ConvTranspose2d(128, 128, 3, 2, 1, 1)
    load_recipe_into(m)
    m = m.cuda()
    x = seeded_randn(*[int(v) for v in g["in0_shape"]], seed=int(g["in0_seed"]))
    xd = to_dev(x, dtype)
    y = m(xd)
    gen = torch.Generator().manual_seed(29)
    gout = torch.randn(y.shape, generator=gen)
    y.backward(gout.to("cuda", dtype))
    tol = TOL[dtype]
    assert_close(y.float(), g["out0"], **tol, what="y")
    assert_close(xd.grad.float(), g["gin0"], **tol, what="dx")
    ref = dict(zip([str(k) for k in g["param_grad_norms_keys"]], g["param_grad_norms"]))
    assert abs(float(m.weight.grad.norm()) - ref["weight"]) <= tol["rtol"] * ref["weight"]
    assert abs(float(m.bias.grad.norm()) - ref["bias"]) <= tol["rtol"] * ref["bias"]


@pytest.mark.parametrize("S,K", [(64, 16), (40, 32), (1280, 64), (1000, 64)])
def test_stem_from_image(S, K):
    """model.0 Conv(3, K, 3, 2) through the stem kernels (fp32 NCHW image in, bf16 compute) against the generic
    path (image_to_nhwc + implicit GEMM): pre-BN output, BN statistics (via the BN'd output), weight gradient.
    1280 / 1000 (the l-scale configs[4] width) take the column-segmented weight-gradient plan."""
    from adrefine import kernels as Kn
    from adrefine.nn.modules import Conv
    torch.manual_seed(0)
    m = Conv(3, K, 3, 2).cuda().train()
    img = torch.rand(2, 3, S, S, device="cuda")
    gout = torch.randn(2, K, S // 2, S // 2, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ya = m.forward_image(img)
    ya.backward(gout)
    ga = m.conv.weight.grad.clone()
    m.conv.weight.grad = None
    yb = m(Kn.image_to_nhwc(img, torch.bfloat16, cpad=8))
    yb.backward(gout)
    gb = m.conv.weight.grad.clone()
    d = (ya.float() - yb.float()).abs().max() / yb.float().abs().max()
    assert float(d) < 2e-2, float(d)
    dg = (ga - gb).norm() / gb.norm()
    assert float(dg) < 1e-2, float(dg)


@pytest.mark.parametrize("shape,k,pad", [((8, 64, 40, 1), (7, 1), (3, 0)), ((8, 64, 1, 40), (1, 7), (0, 3)),
                                         ((4, 32, 20, 12), (5, 3), (2, 1))])
def test_conv_anisotropic_pad_bf16(shape, k, pad):
    """ELA_HSFPN's Conv1d(7) over the pooled (H x 1) / (1 x W) strips (block.py:1413-1416) runs on the bf16 engine
    with separate row / column paddings: forward, input gradient and weight gradient vs torch's fp32 conv on the
    same bf16 operands."""
    import torch.nn.functional as F
    from adrefine import kernels as K
    torch.manual_seed(0)
    N, C, H, W = shape
    x = torch.randn(shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, *k, device="cuda") * 0.05).to(torch.bfloat16).float().requires_grad_(True)
    xd = x.clone().requires_grad_(True)
    y, _ = K.conv2d(xd, w, None, 1, pad)
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(g)
    xr = x.float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 1, pad)
    yr.backward(g.float())
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
    assert rel(y, yr) < 1e-2 and rel(xd.grad, xr.grad) < 1e-2 and rel(w.grad, wr.grad) < 1e-2, \
        (rel(y, yr), rel(xd.grad, xr.grad), rel(w.grad, wr.grad))


@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("c1,c2,k,s,hw", [(16, 32, 3, 2, 24), (32, 64, 1, 1, 20), (64, 128, 3, 1, 13),
                                           (128, 256, 3, 2, 20), (48, 16, 1, 1, 9), (64, 64, 3, 1, 16),
                                           (64, 128, 3, 1, 24), (32, 64, 3, 1, 40), (64, 32, 3, 1, 16),
                                           (128, 192, 1, 1, 10)])
def test_conv_bn_act_eval_fused(act, c1, c2, k, s, hw):
    """Inference Conv-BN-act in one launch (adr_conv2d_fwd_bf16_act; conv_bf16_act_kernel / conv3_act_kernel):
    against a torch fp32 Conv2d -> BatchNorm2d(eval) -> SiLU on the same bf16-rounded operands (bound: 1.5 % of the
    output's max |value|, a few bf16 ulps) and against the unfused HIP pair (conv, then BN + act on the bf16
    conv output), also written into a concat slice through out=."""
    import adrefine.kernels as K
    from adrefine.nn.modules import Conv
    torch.manual_seed(0)
    m = Conv(c1, c2, k, s, act=act)
    load_recipe_into(m)
    with torch.no_grad():  # non-trivial running statistics
        m.bn.running_mean.copy_(torch.randn(c2) * 0.3)
        m.bn.running_var.copy_(torch.rand(c2) * 2 + 0.2)
    m = m.cuda().eval()
    x = seeded_randn(2, c1, hw, hw, seed=7).to("cuda", torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x)
        K.EVAL_CONV_BN_ACT = False
        try:
            y_pair = m(x)
        finally:
            K.EVAL_CONV_BN_ACT = True
        buf = torch.zeros(2, *y.shape[2:], c2 + 16, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
        y_out = m(x, out=buf[:, 8:8 + c2])
        ref = torch.nn.functional.conv2d(x.float(), m.conv.weight.to(torch.bfloat16).float(), None, s, k // 2)
        ref = torch.nn.functional.batch_norm(ref, m.bn.running_mean, m.bn.running_var, m.bn.weight, m.bn.bias,
                                             False, 0.0, m.bn.eps)
        if act:
            ref = torch.nn.functional.silu(ref)
    scale = float(ref.abs().max())
    err = float((y.float() - ref).abs().max()) / scale
    err_pair = float((y.float() - y_pair.float()).abs().max()) / scale
    assert err <= 0.015 and err_pair <= 0.02, (err, err_pair)
    assert torch.equal(y_out, y) and torch.equal(buf[:, 8:8 + c2], y)
    assert float(buf[:, :8].abs().max()) == 0 and float(buf[:, 8 + c2:].abs().max()) == 0


@pytest.mark.parametrize("c1,c2", [(64, 64), (32, 128), (128, 64), (16, 16), (128, 256), (48, 24), (96, 32), (256, 64),
                                   (192, 128), (256, 16)])
def test_conv1_streaming_bf16(c1, c2):
    """1x1 Conv-BN-SiLU on the streaming 1x1 kernel (adr_conv.hip conv1_kernel: weights resident in LDS, the next
    128-row tile prefetched, stats rows per block group) at a size where blocks walk several row tiles (32 x 80^2
    rows), forward (y + BN statistics) and data gradient, against torch fp32 on the same bf16 operands."""
    from adrefine.nn.modules import Conv
    m = Conv(c1, c2, 1, 1)
    rec = load_recipe_into(m)
    m = m.cuda().train()
    x = seeded_randn(32, c1, 80, 80, seed=15)
    xd = to_dev(x, torch.bfloat16)
    y = m(xd)
    g = seeded_randn(*y.shape, seed=16)
    y.backward(g.to("cuda", torch.bfloat16))
    xb = x.bfloat16().float().requires_grad_(True)
    conv = torch.nn.Conv2d(c1, c2, 1, bias=False)
    conv.weight.data = rec["conv.weight"].bfloat16().float()
    bn = torch.nn.BatchNorm2d(c2, eps=1e-3, momentum=0.03)
    bn.weight.data, bn.bias.data = rec["bn.weight"].clone(), rec["bn.bias"].clone()
    bn.running_mean.data, bn.running_var.data = rec["bn.running_mean"].clone(), rec["bn.running_var"].clone()
    yr = torch.nn.functional.silu(bn(conv(xb)))
    yr.backward(g.bfloat16().float())
    rel = lambda a, b: float((a.float().cpu() - b).norm() / (b.norm() + 1e-30))  # noqa: E731
    assert rel(y, yr.detach()) < 1e-2, rel(y, yr.detach())
    assert rel(xd.grad, xb.grad) < 2e-2, rel(xd.grad, xb.grad)
    assert rel(m.conv.weight.grad, conv.weight.grad) < 2e-2
    assert rel(m.bn.running_mean, bn.running_mean) < 1e-2 and rel(m.bn.running_var, bn.running_var) < 1e-2


@pytest.mark.parametrize("act", ["sigmoid", "relu"])
@pytest.mark.parametrize("c1,c2,hw", [(256, 128, 40), (64, 64, 20), (8, 128, 60), (128, 64, 13)])
def test_conv_act_train_fused(act, c1, c2, hw):
    """Training conv + bias + sigmoid / relu in one launch (K.conv_act: the activation on the fp32 accumulator in
    the conv epilogue; backward forms the pre-activation gradient from the saved output, as torch's
    sigmoid_backward / threshold_backward) against torch fp32 on the same bf16 operands: output within 1.5 % of
    max |y|, dx / dw / db within 3 % of their max |value|; and against the unfused HIP pair (conv, then act)."""
    import adrefine.kernels as K
    torch.manual_seed(0)
    w = (torch.randn(c2, c1, 1, 1) / c1 ** 0.5).cuda().requires_grad_()
    b = (torch.randn(c2) * 0.5).cuda().requires_grad_()
    x0 = seeded_randn(2, c1, hw, hw, seed=3).to("cuda", torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dz = seeded_randn(2, c2, hw, hw, seed=4).to("cuda", torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(fuse):
        K.CONV_ACT_FUSE = fuse
        try:
            x = x0.clone().requires_grad_()
            w.grad = b.grad = None
            y = K.conv_act(x, w, b, 1, 0, act)
            y.backward(dz)
            return y.detach().float(), x.grad.float(), w.grad.clone(), b.grad.clone()
        finally:
            K.CONV_ACT_FUSE = True

    yf, dxf, dwf, dbf = run(True)
    yu, dxu, dwu, dbu = run(False)
    xr = x0.float().requires_grad_()
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    br = b.detach().clone().requires_grad_()
    pre = torch.nn.functional.conv2d(xr, wr, br)
    yr = torch.sigmoid(pre) if act == "sigmoid" else torch.relu(pre)
    yr.backward(dz.float())

    def rel(a, r):
        return float((a - r).abs().max()) / max(float(r.abs().max()), 1e-6)

    assert rel(yf, yr.detach()) <= 0.015 and rel(yf, yu) <= 0.02
    for got, pair, ref in ((dxf, dxu, xr.grad), (dwf, dwu, wr.grad), (dbf, dbu, br.grad)):
        assert rel(got, ref) <= 0.03 and rel(got, pair) <= 0.03, (rel(got, ref), rel(got, pair))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("C,hw", [(128, 40), (64, 20), (24, 9)])
def test_mul_pixel(dtype, C, hw):
    """K.mul_pixel (AYHead cls_e * cls_prob, head.py:1170-1172): x * p[:, 0:1] and its backward (dx = dout * p,
    dp[:, 0] = sum_c dout * x, the other channels of dp zero), 16-byte vector path (C = 128 / 64) and the scalar
    path (C = 24), against torch on the same operands; dp written without a prior memset."""
    import adrefine.kernels as K
    x0 = seeded_randn(2, C, hw, hw, seed=1).to("cuda", dtype).contiguous(memory_format=torch.channels_last)
    p0 = seeded_randn(2, 8, hw, hw, seed=2).to("cuda", dtype).contiguous(memory_format=torch.channels_last)
    d0 = seeded_randn(2, C, hw, hw, seed=3).to("cuda", dtype).contiguous(memory_format=torch.channels_last)
    x, p = x0.clone().requires_grad_(), p0.clone().requires_grad_()
    y = K.mul_pixel(x, p)
    y.backward(d0)
    xr, pr = x0.float().requires_grad_(), p0.float().requires_grad_()
    yr = xr * pr[:, 0:1]
    yr.backward(d0.float())
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    for got, ref in ((y, yr), (x.grad, xr.grad), (p.grad, pr.grad)):
        err = float((got.float() - ref.detach()).abs().max()) / max(float(ref.abs().max()), 1e-6)
        assert err <= tol, err
    assert float(p.grad[:, 1:].abs().max()) == 0.0


@pytest.mark.parametrize("c1,c2,n,hw", [(128, 128, 16, 128), (256, 128, 8, 160), (128, 256, 16, 96)])
def test_conv3_wide_tile_bf16(c1, c2, n, hw):
    """The wide 256-pixel x 128-channel 3x3 tile (conv3w_kernel: big-channel convs with >= 512 tiles; l-scale
    shapes) in the forward and the data gradient, with the BN partial statistics, vs torch fp32 on the same bf16
    operands, and against the 128 x 64 halo-tile kernel it replaces (ADR_CONV3W is read once per process, so the
    reference here is torch)."""
    from adrefine import kernels as K
    from adrefine.native import lib
    torch.manual_seed(11)
    x = (torch.randn(n, c1, hw, hw, device="cuda")).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(c2, c1, 3, 3, device="cuda") * (1.0 / (9 * c1) ** 0.5)
    d, _, _ = K.conv_desc(n, hw, hw, c1, c1, c2, 3, 3, 1, 1, 1, 1, c2, torch.bfloat16)
    assert "conv3w" in K._conv2_symbol(d, False) and "conv3w" in K._conv2_symbol(d, True), \
        "the wide tile should take this shape (forward and data gradient)"
    xx = x.detach().clone().requires_grad_(True)
    y, st = K.conv2d(xx, w, None, 1, 1, want_stats=True)
    g = torch.randn_like(y.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(g)
    xr = x.float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, w.to(torch.bfloat16).float(), None, 1, 1)
    yr.backward(g.float())
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
    assert rel(y, yr) < 1e-2, rel(y, yr)
    assert rel(xx.grad, xr.grad) < 1e-2, rel(xx.grad, xr.grad)
    # BN partial statistics: per-tile rows of (sum, sum of squares) of the stored bf16 outputs
    tiles = lib.adr_conv2d_fwd_bf16_stat_tiles(K.ctypes.byref(d))
    s = st.view(tiles, 2, c2).double().sum(0)
    yf = y.detach().double()
    assert torch.allclose(s[0], yf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    assert torch.allclose(s[1], (yf * yf).sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
