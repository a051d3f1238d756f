"""Depthwise conv (adr_dwconv_fwd / adr_dwconv_bwd: the C2PTSSA / EDFFN / Mona depthwise convs, block.py:2376-2710,
mona.py:5-65) against torch's grouped conv in fp32 on the same operands: output, input gradient, weight and bias
gradients, for the whole-image sliding-window kernels (20x20 maps, k 3/5/7) and the direct kernels (larger maps)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,C,H,W,k", [(4, 128, 20, 20, 7), (3, 64, 20, 20, 3), (2, 48, 17, 13, 5), (2, 256, 10, 10, 7),
                                       (2, 32, 40, 40, 3)])
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
