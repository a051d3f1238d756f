"""Depthwise conv (adr_dwconv_fwd / adr_dwconv_bwd: the C2PTSSA / EDFFN / Mona depthwise convs, block.py:2376-2710,
mona.py:5-65) against torch's grouped conv in fp32 on the same operands: output, input gradient, weight and bias
gradients, for the whole-image sliding-window kernels (20x20 maps, k 3/5/7) and the direct kernels (larger maps)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
# (2, 64, 40, 40, 7) / (1, 16, 44, 36, 5): the l-scale C2PTSSA maps, whose 16-channel (bf16) / 8-channel (fp32) image
# slab and 8-channel weight-gradient slab exceed 64 KB of LDS -> the half-width slabs of the whole-image kernels
@pytest.mark.parametrize("N,C,H,W,k", [(4, 128, 20, 20, 7), (3, 64, 20, 20, 3), (2, 48, 17, 13, 5), (2, 256, 10, 10, 7),
                                       (2, 32, 40, 40, 3), (2, 64, 40, 40, 7), (1, 16, 44, 36, 5)])
def test_dwconv_vs_torch(dtype, N, C, H, W, k):
    from adrefine import kernels as K
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, 1, k, k, device="cuda") * 0.2).requires_grad_(True)
    b = (torch.randn(C, device="cuda") * 0.1).requires_grad_(True)
    xd = x.clone().requires_grad_(True)
    y = K.dwconv(xd, w, b, k)
    g = torch.randn(y.shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    y.backward(g)
    xr = x.float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, 1, k // 2, groups=C)
    yr.backward(g.float())
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())  # noqa: E731
    assert rel(y, yr) < tol, rel(y, yr)
    assert rel(xd.grad, xr.grad) < tol, rel(xd.grad, xr.grad)
    assert rel(w.grad, wr.grad) < tol, rel(w.grad, wr.grad)
    assert rel(b.grad, br.grad) < tol, rel(b.grad, br.grad)


@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("c,k,hw", [(64, 3, 20), (128, 3, 40), (256, 5, 20), (32, 7, 16)])
def test_dwconv_bn_act_eval_fused(act, c, k, hw):
    """Inference DWConv-BN-act in one launch (adr_dwconv_fwd_act) against a torch fp32 depthwise Conv2d ->
    BatchNorm2d(eval) -> SiLU on the same bf16 operands (bound: 1.5 % of max |y|) and against the unfused HIP
    pair (depthwise conv, then BN + act: 2 %)."""
    import adrefine.kernels as K
    from adrefine.nn.modules import Conv
    from gpu_util import load_recipe_into
    from recipe import seeded_randn
    torch.manual_seed(1)
    m = Conv(c, c, k, 1, g=c, act=act)
    load_recipe_into(m)
    with torch.no_grad():
        m.bn.running_mean.copy_(torch.randn(c) * 0.3)
        m.bn.running_var.copy_(torch.rand(c) * 2 + 0.2)
    m = m.cuda().eval()
    x = seeded_randn(2, c, hw, hw, seed=9).to("cuda", torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x)
        K.EVAL_CONV_BN_ACT = False
        try:
            y_pair = m(x)
        finally:
            K.EVAL_CONV_BN_ACT = True
        ref = torch.nn.functional.conv2d(x.float(), m.conv.weight.float(), None, 1, k // 2, 1, c)
        ref = torch.nn.functional.batch_norm(ref, m.bn.running_mean, m.bn.running_var, m.bn.weight, m.bn.bias,
                                             False, 0.0, m.bn.eps)
        if act:
            ref = torch.nn.functional.silu(ref)
    scale = float(ref.abs().max())
    err = float((y.float() - ref).abs().max()) / scale
    err_pair = float((y.float() - y_pair.float()).abs().max()) / scale
    assert err <= 0.015 and err_pair <= 0.02, (err, err_pair)
