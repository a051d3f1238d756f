"""Training Conv-BN-act fusion on the bf16 engine (XF kernels): the BN-act backward applied while the producing
conv's data gradient stages its operand (adr_conv2d_dgrad_bf16_bnact, dy side-written for the weight gradient)
against the unfused adr_affine_act_bwd + adr_conv2d_dgrad_bf16 pair.

The staged operand is computed with affine_act_bwd_kernel's bf16 arithmetic and the GEMM is unchanged, so dx, the
weight gradient and the BN parameter gradients must be bitwise equal; the geometries cover every data-gradient
path the fused kernels take: 1x1 (implicit GEMM), 3x3 stride 1 on the halo-tile kernel (C, K % 32 == 0) and on the
implicit GEMM (16-channel reductions, odd widths), 3x3 stride 2 (parity classes), odd map sizes, and a dz that is
a channel slice of a wider gradient (Conv writing into a concat)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(m, x, g, fused, out_buf=None):
    from adrefine import kernels as K
    old = K.BN_XF_BWD
    K.BN_XF_BWD = fused
    try:
        xx = x.detach().clone().requires_grad_(True)
        if out_buf is None:
            z = m(xx)
            z.backward(g)
        else:  # write into a channel slice of a wider activation: dz arrives as a strided view
            buf = torch.zeros(out_buf, device="cuda", dtype=x.dtype).contiguous(memory_format=torch.channels_last)
            z = m(xx, out=buf[:, 8:8 + m.conv.out_channels])
            z.backward(g)
        res = (z.detach().clone(), xx.grad.clone(), m.conv.weight.grad.clone(), m.bn.weight.grad.clone(),
               m.bn.bias.grad.clone())
    finally:
        K.BN_XF_BWD = old
        m.zero_grad(set_to_none=True)
    assert not K._BNXF_PENDING, "a pending BN-act backward was never consumed"
    return res


CASES = [  # n, c1, c2, k, s, h, w
    (4, 64, 64, 1, 1, 20, 20),      # 1x1
    (2, 32, 64, 1, 1, 40, 24),      # 1x1, K > C
    (4, 64, 64, 3, 1, 16, 16),      # 3x3 s1 halo tiles (TW 16)
    (2, 32, 32, 3, 1, 24, 8),       # 3x3 s1 halo tiles (TW 8)
    (2, 16, 16, 3, 1, 20, 20),      # 3x3 s1 implicit GEMM (16-channel reduction, tap-packed K-steps)
    (2, 32, 64, 3, 1, 13, 11),      # 3x3 s1 implicit GEMM (odd width)
    (2, 32, 64, 3, 2, 40, 40),      # 3x3 s2 (parity classes)
    (2, 64, 128, 3, 2, 21, 19),     # 3x3 s2, odd sizes, several column tiles
    (2, 128, 256, 3, 2, 20, 20),    # wide reduction (256 BN channels)
]


@pytest.mark.parametrize("n,c1,c2,k,s,h,w", CASES)
def test_dgrad_bnact_matches_unfused(n, c1, c2, k, s, h, w):
    from adrefine.nn.modules.conv import Conv
    torch.manual_seed(0)
    m = Conv(c1, c2, k, s).cuda().train()
    with torch.no_grad():
        m.bn.weight.uniform_(0.5, 1.5)
        m.bn.bias.uniform_(-0.3, 0.3)
    x = (torch.randn(n, c1, h, w, device="cuda") * 1.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
    g = torch.randn(n, c2, ho, wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = _run(m, x, g, True)
    b = _run(m, x, g, False)
    for name, u, v in zip(("z", "dx", "dw", "dgamma", "dbeta"), a, b):
        assert torch.equal(u, v), (name, float((u.float() - v.float()).abs().max()))


def test_dgrad_bnact_strided_dz():
    """The conv writes its activation into a channel slice of a wider buffer (C2f / SPPF concat), so the upstream
    gradient dz is a strided view (channel stride 80, offset 8)."""
    from adrefine.nn.modules.conv import Conv
    torch.manual_seed(0)
    m = Conv(32, 64, 3, 1).cuda().train()
    x = torch.randn(2, 32, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = _run(m, x, g, True, out_buf=(2, 80, 16, 16))
    b = _run(m, x, g, False, out_buf=(2, 80, 16, 16))
    for name, u, v in zip(("z", "dx", "dw", "dgamma", "dbeta"), a, b):
        assert torch.equal(u, v), (name, float((u.float() - v.float()).abs().max()))


def test_dgrad_bnact_whole_net_step():
    """One bf16 train step of the 701 graph at 320^2 bs 2: fused and unfused backward give the same loss and
    bitwise-equal parameter gradients (every Conv of the net runs through BnXf)."""
    from adrefine import kernels as K
    from adrefine.nn.tasks import DetectionModel
    from conftest import ROOT
    from gpu_util import load_recipe_into
    from recipe import synthetic_images
    torch.manual_seed(0)
    m = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16)
    load_recipe_into(m)
    m = m.cuda().train()
    img = synthetic_images(2, 320, seed=3).cuda()
    batch = {"img": img, "batch_idx": torch.tensor([0., 0., 1.]), "cls": torch.tensor([[1.], [5.], [7.]]),
             "bboxes": torch.tensor([[0.5, 0.5, 0.3, 0.4], [0.2, 0.3, 0.1, 0.2], [0.6, 0.6, 0.5, 0.3]])}
    grads = []
    for fused in (True, False):
        old = K.BN_XF_BWD
        K.BN_XF_BWD = fused
        try:
            sd = {k: v.clone() for k, v in m.state_dict().items()}
            loss, _ = m(batch)
            loss.backward()
            grads.append((float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
            m.zero_grad(set_to_none=True)
            m.load_state_dict(sd)  # BN running statistics back
        finally:
            K.BN_XF_BWD = old
    (la, ga), (lb, gb) = grads
    assert la == lb
    assert set(ga) == set(gb)
    bad = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not bad, bad[:10]
