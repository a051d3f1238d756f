"""GroupNorm + activation fused per image (adr_gn_act_fused / adr_gn_act_bwd_fused / adr_gn_param_grad) against
torch.nn.functional.group_norm + the activation in fp32 (forward, input gradient, gamma / beta gradients), on the
AYHead map sizes and ELA's pooled (H x 1) strips, and against the three-launch path it replaces."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ACTS = {"silu": F.silu, "sigmoid": torch.sigmoid, "none": lambda v: v}


def _run(x, gn, act, fused):
    from adrefine import kernels as K
    old, oldhw = K._GN_FUSED, K._GN_FUSED_MAXHW
    K._GN_FUSED, K._GN_FUSED_MAXHW = fused, 1 << 30
    try:
        xx = x.detach().clone().requires_grad_(True)
        z = K.gn_act(xx, gn, act)
        torch.manual_seed(1)  # the same upstream gradient for every path
        g = torch.randn_like(z.float()).to(z.dtype).contiguous(memory_format=torch.channels_last)
        z.backward(g)
        return z, xx.grad, gn.weight.grad.clone(), gn.bias.grad.clone(), g
    finally:
        K._GN_FUSED, K._GN_FUSED_MAXHW = old, oldhw
        gn.weight.grad = gn.bias.grad = None


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,act", [((4, 64, 20, 20), "silu"), ((2, 64, 80, 80), "silu"), ((3, 128, 40, 40), "none"),
                                       ((4, 32, 25, 1), "sigmoid"), ((2, 256, 10, 10), "silu")])
def test_gn_fused_vs_torch(dtype, shape, act):
    torch.manual_seed(0)
    N, C, H, W = shape
    gn = torch.nn.GroupNorm(16, C).cuda()
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(shape, device="cuda") * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    z, dx, dgw, dgb, g = _run(x, gn, act, True)
    xr = x.detach().float().requires_grad_(True)
    wr = gn.weight.detach().clone().requires_grad_(True)
    br = gn.bias.detach().clone().requires_grad_(True)
    zr = ACTS[act](F.group_norm(xr, 16, wr, br, gn.eps))
    zr.backward(g.float())
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-12))  # noqa: E731
    assert rel(z, zr) < tol, rel(z, zr)
    assert rel(dx, xr.grad) < 2 * tol, rel(dx, xr.grad)
    assert rel(dgw, wr.grad) < 2 * tol, rel(dgw, wr.grad)
    assert rel(dgb, br.grad) < 2 * tol, rel(dgb, br.grad)
    # and the three-launch path (nc_reduce + gn_finalize + affine_act) agrees
    z2, dx2, dgw2, dgb2, _ = _run(x, gn, act, False)
    assert rel(z, z2.float()) < tol and rel(dx, dx2.float()) < 2 * tol and rel(dgw, dgw2) < 2 * tol
