"""The stride-2 3x3 data gradient on super-pixel halo tiles (adr_conv.hip dg2_kernel, DG2H): every parity class of
the dx tile from one staged dy halo and one 9-tap weight slab per 32-channel chunk. Reference: the data gradient of
nn.Conv2d(k3, s2, p1) (Conv.forward, nn/modules/conv.py:48-50) = conv_transpose2d(dy, w, stride 2, padding 1,
output_padding (H + 1) % 2), checked against torch fp32 on the same bf16 operands; the accumulate / addend epilogue
forms against the plain result. Shapes: one (C = 16, 32) and two / three column tiles (C = 128, 48), odd dx sizes
(ragged super-pixel tiles and a class-(1, .) row with no dy below it), dy channels 32..256."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


CASES = [  # n, C (dx channels), K (dy channels), H, W
    (2, 16, 32, 40, 40),
    (2, 64, 64, 32, 32),
    (2, 128, 128, 20, 20),
    (2, 48, 32, 18, 18),
    (2, 32, 64, 21, 19),
    (1, 64, 256, 6, 6),
    (4, 64, 128, 80, 80),
]


@pytest.mark.parametrize("n,C,Kc,H,W", CASES)
def test_dg2_matches_conv_transpose(n, C, Kc, H, W, monkeypatch):
    from adrefine import kernels as K
    monkeypatch.setenv("ADR_DG2H", "2")  # DG2H even where the plan would pick the per-class GEMM (ragged tiles)
    from adrefine.native import lib
    torch.manual_seed(3)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = _nhwc(torch.randn(n, Kc, Ho, Wo, device="cuda").to(torch.bfloat16))
    w = (torch.randn(Kc, C, 3, 3, device="cuda") * (1.0 / (9 * Kc) ** 0.5)).to(torch.bfloat16).float()
    _, crsk = K.pack_weight2(w, torch.bfloat16)
    d, _, _ = K.conv_desc(n, H, W, C, C, Kc, 3, 3, 2, 2, 1, 1, Kc, torch.bfloat16)
    assert "dg2_kernel" in K._conv2_symbol(d, True), K._conv2_symbol(d, True)
    dx = K.empty_act(n, C, H, W, torch.bfloat16, "cuda")
    lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(crsk.data_ptr()),
                              None, ctypes.c_void_p(dx.data_ptr()), 0, K.stream())
    ref = torch.nn.functional.conv_transpose2d(dy.float(), w, None, 2, 1, output_padding=(H + 1) % 2)
    assert ref.shape == dx.shape
    rel = float((dx.float() - ref).norm() / ref.norm())
    err = float((dx.float() - ref).abs().max() / ref.abs().max())
    assert rel < 5e-3 and err < 1e-2, (rel, err)
    # accumulate and addend forms: dx2 = dx + dgrad (+ addend) in one rounding
    add = _nhwc(torch.randn(n, C, H, W, device="cuda").to(torch.bfloat16))
    dx2 = dx.clone()
    lib.adr_conv2d_dgrad_bf16_add(ctypes.byref(d), ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(crsk.data_ptr()),
                                  ctypes.c_void_p(dx2.data_ptr()), 1, ctypes.c_void_p(add.data_ptr()), C, K.stream())
    want = (dx.float() + ref + add.float())
    rel2 = float((dx2.float() - want).norm() / want.norm())
    assert rel2 < 5e-3, rel2


def test_dg2_plan_padding_rule(monkeypatch):
    """Default plan: DG2H only where its 8 x 8 super-pixel tiles cover the dy grid with <= 15 % padding (80^2 -> 40^2
    yes, 20^2 -> 10^2 no: the per-class implicit GEMM runs those)."""
    from adrefine import kernels as K
    monkeypatch.setenv("ADR_DG2H", "1")
    d, _, _ = K.conv_desc(2, 80, 80, 64, 64, 128, 3, 3, 2, 2, 1, 1, 128, torch.bfloat16)
    assert "dg2_kernel" in K._conv2_symbol(d, True)
    d, _, _ = K.conv_desc(2, 20, 20, 64, 64, 128, 3, 3, 2, 2, 1, 1, 128, torch.bfloat16)
    assert "conv_bf16_kernel" in K._conv2_symbol(d, True)


def test_dg2_concat_slice_output(monkeypatch):
    """dx written into a channel slice of a wider gradient buffer (the concat-gradient sink): channel stride 96,
    offset 32; the other channels untouched."""
    from adrefine import kernels as K
    monkeypatch.setenv("ADR_DG2H", "2")
    from adrefine.native import lib
    torch.manual_seed(4)
    n, C, Kc, H, W = 2, 32, 64, 24, 24
    dy = _nhwc(torch.randn(n, Kc, H // 2, W // 2, device="cuda").to(torch.bfloat16))
    w = (torch.randn(Kc, C, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).float()
    _, crsk = K.pack_weight2(w, torch.bfloat16)
    buf = _nhwc(torch.full((n, 96, H, W), 7.0, device="cuda", dtype=torch.bfloat16))
    d, _, _ = K.conv_desc(n, H, W, C, 96, Kc, 3, 3, 2, 2, 1, 1, Kc, torch.bfloat16)
    d.x_coff = 32
    lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(crsk.data_ptr()),
                              None, ctypes.c_void_p(buf.data_ptr()), 0, K.stream())
    ref = torch.nn.functional.conv_transpose2d(dy.float(), w, None, 2, 1, output_padding=1)
    got = buf[:, 32:64].float()
    assert float((got - ref).norm() / ref.norm()) < 5e-3
    assert bool((buf[:, :32] == 7).all()) and bool((buf[:, 64:] == 7).all())
