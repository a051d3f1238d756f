"""In-producer normalisation finalize (adr_norm_fin: adr_conv2d_fwd_bf16_fin, adr_nc_reduce_fin) against the
separate finalize launches it replaces (adr_bn_finalize / adr_bn_bwd_finalize / adr_gn_finalize /
adr_gn_bwd_finalize), and against float64 batch statistics of the stored conv output.

Bounds: the finalize arithmetic is the same double-precision formula; only the order in which the partial rows
are summed differs (two fixed-order levels instead of one strided sum), so the fp32 coefficients agree to a few
ulp: scale / shift / running statistics / mean / rstd within 2e-6 relative, activations within one bf16 ulp of
|z| (8e-3 relative to max |z|) and gradients within 1e-5 relative L2 (fp32) / 2e-2 (bf16, where a 1-ulp coefficient
change can flip the rounding of single elements). The fin path is bitwise repeatable and leaves its arrival
counters at zero."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _conv(c1, c2, k, s, dtype):
    from adrefine.nn.modules.conv import Conv
    torch.manual_seed(0)
    m = Conv(c1, c2, k, s).cuda().train()
    with torch.no_grad():
        m.bn.weight.uniform_(0.5, 1.5)
        m.bn.bias.uniform_(-0.3, 0.3)
        m.bn.running_var.uniform_(0.5, 2.0)
    return m


def _step(m, x, g, fin):
    """One train-mode fwd + bwd with the fin path on / off: (z, dx, dw, dgamma, dbeta, running mean, running var)."""
    from adrefine import kernels as K
    old = K.NORM_FIN
    K.NORM_FIN = fin
    rm, rv = m.bn.running_mean.clone(), m.bn.running_var.clone()
    try:
        xx = x.detach().clone().requires_grad_(True)
        z = m(xx)
        z.backward(g)
        out = (z.detach().float(), xx.grad.float(), m.conv.weight.grad.clone(), m.bn.weight.grad.clone(),
               m.bn.bias.grad.clone(), m.bn.running_mean.clone(), m.bn.running_var.clone())
    finally:
        K.NORM_FIN = old
        m.zero_grad(set_to_none=True)
        with torch.no_grad():
            m.bn.running_mean.copy_(rm)
            m.bn.running_var.copy_(rv)
    return out


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


def _counters_zero():
    from adrefine import kernels as K
    for cnt, _ in K._FIN_POOLS.values():
        assert int(cnt.abs().sum()) == 0, "arrival counters not reset"


# geometries: 1x1 (conv_bf16 engine), 3x3 s1 (conv3 halo tiles), 3x3 s2 (implicit GEMM), a wide 1x1 with several
# column tiles, and maps large enough for the two-level reduction (P > 128 row tiles)
SHAPES = [(4, 64, 64, 1, 1, 20), (4, 64, 64, 3, 1, 20), (2, 32, 64, 3, 2, 80), (2, 128, 256, 1, 1, 40),
          (8, 64, 32, 1, 1, 80), (4, 32, 32, 3, 1, 160)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,c1,c2,k,s,hw", SHAPES)
def test_conv_bn_fin_matches_separate_finalize(dtype, n, c1, c2, k, s, hw):
    m = _conv(c1, c2, k, s, dtype)
    torch.manual_seed(1)
    x = (torch.randn(n, c1, hw, hw, device="cuda") * 1.5 + 0.2).to(dtype).contiguous(memory_format=torch.channels_last)
    ho = (hw + 2 * (k // 2) - k) // s + 1
    g = torch.randn(n, c2, ho, ho, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    a = _step(m, x, g, True)
    _counters_zero()
    b = _step(m, x, g, False)
    z, zr = a[0], b[0]
    assert float((z - zr).abs().max()) <= 8e-3 * float(zr.abs().max()) + 1e-6
    gtol = 1e-5 if dtype == torch.float32 else 2e-2
    for name, u, v in zip(("dx", "dw", "dgamma", "dbeta"), a[1:5], b[1:5]):
        assert _rel(u, v) < gtol, (name, _rel(u, v))
    for name, u, v in zip(("running_mean", "running_var"), a[5:], b[5:]):
        assert float(((u - v).abs() / (v.abs() + 1e-6)).max()) < 2e-6, name
    # repeatable bit for bit (fixed-order sums whichever workgroup finishes last)
    c = _step(m, x, g, True)
    for u, v in zip(a, c):
        assert torch.equal(u, v)


@pytest.mark.parametrize("n,c,hw", [(4, 64, 20), (2, 32, 160), (64, 16, 40)])
def test_conv_bn_fin_statistics_vs_float64(n, c, hw):
    """The finalized mean / rstd / scale / shift against float64 statistics of the conv output the kernel stored."""
    from adrefine import kernels as K
    m = _conv(c, c, 1, 1, torch.bfloat16)
    x = torch.randn(n, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fin = K.BnFin(m.bn, x.device)
    rm0 = m.bn.running_mean.clone()
    old = K.NORM_FIN
    K.NORM_FIN = True
    try:
        y, st = K.conv2d(x, m.conv.weight, None, 1, 0, True, 0, bnfin=fin)
    finally:
        K.NORM_FIN = old
    assert fin.done
    yd = y.detach().double()
    mean = yd.mean(dim=(0, 2, 3))
    var = yd.var(dim=(0, 2, 3), unbiased=False)
    rstd = 1.0 / torch.sqrt(var + m.bn.eps)
    assert float(((fin.mean.double() - mean).abs() / (mean.abs() + 1e-3)).max()) < 1e-5
    assert float(((fin.rstd.double() - rstd).abs() / rstd).max()) < 1e-5
    sc = m.bn.weight.double() * rstd
    assert float(((fin.scale.double() - sc).abs() / sc.abs()).max()) < 1e-5
    sh = m.bn.bias.double() - mean * sc
    assert float((fin.shift.double() - sh).abs().max()) < 1e-4
    rm = (1 - m.bn.momentum) * rm0.double() + m.bn.momentum * mean
    assert float((m.bn.running_mean.double() - rm).abs().max()) < 1e-5
    _counters_zero()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dwconv_bn_fin(dtype):
    """BN over a depthwise conv output: statistics + finalize from adr_nc_reduce_fin (BN_FWD / BN_BWD)."""
    from adrefine.nn.modules.conv import DWConv
    torch.manual_seed(0)
    m = DWConv(64, 64, 3).cuda().train()
    x = torch.randn(4, 64, 40, 40, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.randn(4, 64, 40, 40, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    a = _step(m, x, g, True)
    b = _step(m, x, g, False)
    assert float((a[0] - b[0]).abs().max()) <= 8e-3 * float(b[0].abs().max()) + 1e-6
    gtol = 1e-5 if dtype == torch.float32 else 2e-2
    for u, v in zip(a[1:5], b[1:5]):
        assert _rel(u, v) < gtol
    _counters_zero()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 64, 80, 80), (4, 128, 40, 40), (3, 256, 24, 24)])
def test_gn_fin_matches_separate_finalize(dtype, shape):
    """GroupNorm's three-launch path (maps above the per-image fused kernel's threshold) with the per-image
    finalize inside adr_nc_reduce_fin, forward and backward, against adr_gn_finalize / adr_gn_bwd_finalize."""
    from adrefine import kernels as K
    torch.manual_seed(0)
    N, C, H, W = shape
    gn = torch.nn.GroupNorm(16, C).cuda()
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(shape, device="cuda") * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    res = []
    old, oldf = K._GN_FUSED, K.NORM_FIN
    try:
        K._GN_FUSED = False
        for fin in (True, False):
            K.NORM_FIN = fin
            xx = x.detach().clone().requires_grad_(True)
            z = K.gn_act(xx, gn, "silu")
            z.backward(g)
            res.append((z.detach().float(), xx.grad.float(), gn.weight.grad.clone(), gn.bias.grad.clone()))
            gn.weight.grad = gn.bias.grad = None
    finally:
        K._GN_FUSED, K.NORM_FIN = old, oldf
    (z, dx, dgw, dgb), (zr, dxr, dgwr, dgbr) = res
    assert float((z - zr).abs().max()) <= 8e-3 * float(zr.abs().max()) + 1e-6
    gtol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(dx, dxr) < gtol and _rel(dgw, dgwr) < gtol and _rel(dgb, dgbr) < gtol
    _counters_zero()
