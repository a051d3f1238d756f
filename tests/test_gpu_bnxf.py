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


@pytest.fixture(autouse=True)
def _xf_everywhere(monkeypatch):
    """The engine declines the XF data gradient where it measured slower (the per-tile engine instead of the
    streaming 1x1 kernel, DG2H, the 3x3 halo tiles; adr_conv2d_bf16_xf_reuse). Those fused kernels stay correct and tested: take them."""
    monkeypatch.setenv("ADR_XF_STREAM", "1")
    monkeypatch.setenv("ADR_XF_DG2", "1")
    monkeypatch.setenv("ADR_XF_CONV3", "1")


@pytest.fixture(autouse=True)
def _no_bstat():
    """These tests pin the XF fusions bitwise against the unfused pairs. The BN backward statistics taken in the
    consumer's data gradient (BSTAT) sum the same terms in another order — tested on its own in test_gpu_bstat.py —
    so it is off here, where its presence would differ between the two sides."""
    from adrefine import kernels as K
    old = K.BN_BSTAT
    K.BN_BSTAT = False
    yield
    K.BN_BSTAT = old


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


# ---- forward fusion: the consumer conv stages the producer's pre-BN output through the BN-act (BnFwd) ----

def _pair_run(p, q, x, g, fused):
    """q(p(x)) with p's output handed lazily to q (Conv.forward(lazy=True)); returns outputs, input gradient, the
    parameter gradients and p's BN running statistics; the fused and unfused runs start from the same state."""
    from adrefine import kernels as K
    old = K.BN_XF_FWD
    K.BN_XF_FWD = fused
    sd = ({k: v.clone() for k, v in p.state_dict().items()}, {k: v.clone() for k, v in q.state_dict().items()})
    try:
        xx = x.detach().clone().requires_grad_(True)
        z1 = p(xx, lazy=True)
        assert bool(K._BNF_PENDING) == fused
        z2 = q(z1)
        assert not K._BNF_PENDING
        z2.backward(g)
        res = [z2.detach().clone(), z1.detach().clone(), xx.grad.clone()]
        res += [t.grad.clone() for t in (p.conv.weight, p.bn.weight, p.bn.bias, q.conv.weight, q.bn.weight, q.bn.bias)]
        res += [p.bn.running_mean.clone(), p.bn.running_var.clone(), q.bn.running_mean.clone()]
    finally:
        K.BN_XF_FWD = old
        p.zero_grad(set_to_none=True)
        q.zero_grad(set_to_none=True)
        p.load_state_dict(sd[0])
        q.load_state_dict(sd[1])
    return res


FWD_CASES = [  # n, c1, c, k1, s1, k2, h, w : p = Conv(c1, c, k1, s1), q = Conv(c, c, k2)
    (4, 32, 32, 3, 1, 3, 16, 16),    # bottleneck 3x3 -> 3x3 on the halo tiles (TW 16)
    (2, 64, 64, 3, 1, 3, 24, 8),     # halo tiles TW 8, two 32-channel chunks
    (4, 16, 32, 3, 2, 1, 40, 40),    # Conv s2 -> C3k2.cv1 1x1 on the streaming kernel (KT 64)
    (2, 64, 128, 3, 2, 1, 20, 20),   # 1x1 128 -> 128: streaming kernel, two column tiles (KT 128)
    (2, 16, 16, 3, 1, 3, 20, 20),    # 16-channel 3x3: the implicit GEMM would stage x9 -> written first (no fusion)
]


@pytest.mark.parametrize("n,c1,c,k1,s1,k2,h,w", FWD_CASES)
def test_fwd_bnact_matches_unfused(n, c1, c, k1, s1, k2, h, w):
    """Bitwise: the fused forward stages exactly the bf16 values adr_affine_act stores and runs the plain forward's
    tiling, so outputs, the side-written z, every gradient and the running statistics equal the unfused pair's."""
    from adrefine.nn.modules.conv import Conv
    torch.manual_seed(1)
    p = Conv(c1, c, k1, s1).cuda().train()
    q = Conv(c, c, k2, 1).cuda().train()
    with torch.no_grad():
        for m in (p, q):
            m.bn.weight.uniform_(0.5, 1.5)
            m.bn.bias.uniform_(-0.3, 0.3)
    x = (torch.randn(n, c1, h, w, device="cuda") * 1.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ho, wo = (h + 2 * (k1 // 2) - k1) // s1 + 1, (w + 2 * (k1 // 2) - k1) // s1 + 1
    g = torch.randn(n, c, ho, wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = _pair_run(p, q, x, g, True)
    b = _pair_run(p, q, x, g, False)
    names = ("out", "z", "dx", "dw1", "dgamma1", "dbeta1", "dw2", "dgamma2", "dbeta2", "rm1", "rv1", "rm2")
    for name, u, v in zip(names, a, b):
        assert torch.equal(u, v), (name, float((u.float() - v.float()).abs().max()))


def test_fwd_bnact_other_reader_writes_first():
    """A pending BN-act output read by anything but its consumer conv (here a channel slice through an elementwise
    kernel) is written first, so the reader sees the true activation."""
    from adrefine import kernels as K
    from adrefine.nn.modules.conv import Conv
    torch.manual_seed(2)
    p = Conv(32, 32, 3, 1).cuda().train()
    x = torch.randn(2, 32, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    z_ref = p(x).detach().clone()
    z = p(x, lazy=True)
    assert K._BNF_PENDING
    s = K.act(z[:, 8:24], "relu")  # another reader of a view of z
    assert not K._BNF_PENDING
    assert torch.equal(z.detach(), z_ref) and torch.equal(s.detach(), torch.relu(z_ref[:, 8:24]))


def test_fwd_bnact_whole_net_step():
    """One bf16 train step of the 701 graph at 320^2 bs 2 with and without the forward fusion (11 Conv -> Conv
    pairs: the bottlenecks and the Conv layers feeding C3k2 cv1): same loss, bitwise parameter gradients."""
    from adrefine import kernels as K
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
    for fused in (True, False):
        old = K.BN_XF_FWD
        K.BN_XF_FWD = fused
        try:
            sd = {k: v.clone() for k, v in m.state_dict().items()}
            loss, _ = m(batch)
            loss.backward()
            runs.append((float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                         {k: v.clone() for k, v in m.state_dict().items()}))
            m.zero_grad(set_to_none=True)
            m.load_state_dict(sd)
        finally:
            K.BN_XF_FWD = old
    (la, ga, sa), (lb, gb, sb) = runs
    assert la == lb
    bad = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not bad, bad[:10]
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:10]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("sliced", [False, True])
def test_bottleneck_residual_in_bnact_pass(dtype, sliced):
    """Bottleneck's shortcut added in cv2's BN-act pass (adr_affine_act_res) against the BN-act + add pair:
    output, input gradient and every parameter gradient bitwise equal, writing into a concat slot or not."""
    import copy

    from adrefine import kernels as K
    from adrefine.nn.modules.block import Bottleneck
    torch.manual_seed(1)
    m = Bottleneck(64, 64, True, k=(3, 3), e=1.0).cuda().train()
    with torch.no_grad():
        for cv in (m.cv1, m.cv2):
            cv.bn.weight.uniform_(0.5, 1.5)
            cv.bn.bias.uniform_(-0.3, 0.3)
    ref = copy.deepcopy(m)
    x = torch.randn(2, 64, 20, 20, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, 64, 20, 20, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)

    def unfused(mod, xx, out=None):  # the pre-fusion composition: BN-act pass, then the add
        xa, xb = K.fanout(xx)
        return K.add(xa, mod.cv2(mod.cv1(xb, lazy=True)), out=out)

    outs = []
    for mod, fn in ((m, lambda mod, xx, out=None: mod(xx, out=out)), (ref, unfused)):
        xx = x.detach().clone().requires_grad_(True)
        if sliced:
            buf = torch.zeros(2, 128, 20, 20, device="cuda", dtype=dtype).contiguous(memory_format=torch.channels_last)
            z = fn(mod, xx, out=buf[:, 32:96])
        else:
            z = fn(mod, xx)
        z.backward(g)
        torch.cuda.synchronize()
        outs.append((z.detach().clone(), xx.grad.clone(), [p.grad.clone() for p in mod.parameters()]))
    (z0, dx0, p0), (z1, dx1, p1) = outs
    assert torch.equal(z0, z1)
    assert torch.equal(dx0, dx1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))
