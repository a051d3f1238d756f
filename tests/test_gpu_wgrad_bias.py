"""Bias gradients fused into the weight-gradient GEMM (adr_conv2d_wgrad_partials_bias / adr_wgrad_job.bias): the
column sums sum_p dy[p][k] of nn.Conv2d's bias backward (reference nn/modules/conv.py:36-54; the AYHead's biased
convs, head.py) come out of the WGRAD launch that already holds dy in registers. The weight partials must be
bitwise the plain launch's; the split rows summed must match an fp64 column sum of the same bf16 dy (the products
are dy * 1, exact; only the fp32 summation order differs). Shapes cover the generic tile kernel (1x1, 3x3 s2) and
the 3x3 s1 halo-tile kernel (wgrad3, both KF variants)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,H,W,C,K,R,S", [(4, 40, 40, 64, 80, 1, 1), (2, 80, 80, 128, 128, 1, 1),
                                           (4, 40, 40, 64, 128, 3, 2), (1344 // 64, 20, 20, 64, 64, 1, 1),
                                           (4, 80, 80, 128, 128, 3, 1), (3, 20, 20, 64, 32, 3, 1)])
def test_wgrad_bias_partials(N, H, W, C, K, R, S):
    from adrefine import kernels as Kn
    from adrefine.native import lib
    torch.manual_seed(0)
    pad = R // 2
    x = _nhwc(torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16))
    d, Ho, Wo = Kn.conv_desc(N, H, W, C, C, K, R, R, S, S, pad, pad, K, torch.bfloat16)
    dy = _nhwc(torch.randn(N, K, Ho, Wo, device="cuda").to(torch.bfloat16))
    assert lib.adr_conv2d_wgrad_bias_fusable(ctypes.byref(d)) == 1
    splits = lib.adr_conv2d_wgrad_splits(ctypes.byref(d))
    n = splits * K * R * R * C
    wa = torch.empty(n, device="cuda")
    wb = torch.empty(n, device="cuda")
    bp = torch.full((splits * 2 * K,), float("nan"), device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.adr_conv2d_wgrad_partials(ctypes.byref(d), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(dy.data_ptr()),
                                         ctypes.c_void_p(wa.data_ptr()), 0, st) == 0
    assert lib.adr_conv2d_wgrad_partials_bias(ctypes.byref(d), ctypes.c_void_p(x.data_ptr()),
                                              ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(wb.data_ptr()),
                                              ctypes.c_void_p(bp.data_ptr()), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(wa, wb)
    rows = bp.view(splits, 2, K)[:, 0]
    assert torch.isfinite(rows).all()
    got = rows.double().sum(0)
    ref = dy.double().sum((0, 2, 3))
    assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) + 1e-6


def test_wgrad_bias_train_step_matches_unfused(monkeypatch):
    """fwd + loss + bwd of the 701 model (bf16, 320^2, bs 4) into the trainer's gradient arena: every bias gradient
    with the fused column sums vs the separate column-sum pass (ADR_FUSE_WG_BIAS=0), same weights and batch; every
    other gradient bitwise unchanged."""
    from pathlib import Path
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.data.synthetic import train_batch
    from adrefine.nn.tasks import DetectionModel
    root = Path(__file__).resolve().parents[1]
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("ADR_FUSE_WG_BIAS", mode)
        torch.manual_seed(0)
        m = DetectionModel(str(root / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"),
                           compute_dtype=torch.bfloat16).cuda()
        tr = FusedTrainer(m, batch_size=4)
        batch, _ = train_batch(4, 320, seed=0, device="cuda")
        tr.forward_backward(tr._prepare(batch))
        torch.cuda.synchronize()
        out[mode] = {name: tr.grad[off:off + p.numel()].clone()
                     for (name, p, _, isp), off in zip(tr.entries, tr._goff) if isp}
    nb = 0
    for k in out["0"]:
        a, b = out["0"][k], out["1"][k]
        if k.endswith("bias"):
            nb += 1
            assert float((a - b).abs().max()) <= 1e-4 * float(a.abs().max()) + 1e-7, k
        else:
            assert torch.equal(a, b), k
    assert nb > 0


@pytest.mark.parametrize("N,H,W,C,K,R,S", [(2, 80, 80, 128, 128, 1, 1), (4, 40, 40, 256, 136, 3, 2),
                                           (3, 17, 13, 192, 160, 1, 1), (2, 9, 7, 136, 200, 3, 2)])
def test_wgrad_double_buffered_tile_bitwise(monkeypatch, N, H, W, C, K, R, S):
    """The 128 x 128 WGRAD tile runs double-buffered (two LDS stages, loads two k-steps ahead, adr_wgrad.hip
    wgrad_bf16_body<.., DB>): same k-steps, same order, so its weight partials and fused bias rows must be bitwise
    the single-stage kernel's (ADR_WG_DB=0) — including ragged k-steps (split ends inside a step), channel tails and
    the 3x3 stride-2 gathers."""
    from adrefine import kernels as Kn
    from adrefine.native import lib
    torch.manual_seed(1)
    pad = R // 2
    x = _nhwc(torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16))
    d, Ho, Wo = Kn.conv_desc(N, H, W, C, C, K, R, R, S, S, pad, pad, K, torch.bfloat16)
    dy = _nhwc(torch.randn(N, K, Ho, Wo, device="cuda").to(torch.bfloat16))
    assert lib.adr_conv2d_wgrad_batched_tile(ctypes.byref(d)) == 128 * 256 + 128
    splits = lib.adr_conv2d_wgrad_splits(ctypes.byref(d))
    n = splits * K * R * R * C
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("ADR_WG_DB", mode)
        w = torch.full((n,), float("nan"), device="cuda")
        bp = torch.full((splits * 2 * K,), float("nan"), device="cuda")
        assert lib.adr_conv2d_wgrad_partials_bias(ctypes.byref(d), ctypes.c_void_p(x.data_ptr()),
                                                  ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                                                  ctypes.c_void_p(bp.data_ptr()), st) == 0
        torch.cuda.synchronize()
        out[mode] = (w, bp.view(splits, 2, K)[:, 0].clone())
    assert torch.isfinite(out["1"][0]).all()
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])
    ref = torch.einsum("nkhw,nchw->kc", dy.float(), x.float()) if R == 1 else None
    if ref is not None:
        got = out["1"][0].view(splits, K, C).sum(0)
        assert float((got - ref).abs().max()) <= 1e-4 * float(ref.abs().max())
