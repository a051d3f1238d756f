"""Concurrent AYHead levels (kernels.run_levels: one stream per pyramid level, forward and backward; gradient slabs
of the shared head parameters folded into the arena in the serial accumulation order). The reference loops the
levels serially (head.py:1132); the concurrent path must be BITWISE the serial one (ADR_LEVEL_STREAMS=0):
the whole gradient arena after a backward, the parameters / EMA / BN running statistics after optimizer steps, the
loss items, eagerly and through captured hipGraphs, in fp32 parity mode and in bf16; and the eval forward."""
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _model(dtype):
    from adrefine.nn.tasks import DetectionModel
    from gpu_util import load_recipe_into
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


def _run(dtype, levels, graph, bs=4, img=320):
    from adrefine import kernels as K
    from adrefine.data.synthetic import train_batch
    from adrefine.engine.trainer import FusedTrainer
    old = K.LEVEL_STREAMS
    K.LEVEL_STREAMS = levels
    try:
        m = _model(dtype)
        tr = FusedTrainer(m, batch_size=bs, nbs=bs)
        b0, _ = train_batch(bs, img, seed=3, device="cuda", u8=True)
        b1, _ = train_batch(bs, img, seed=4, device="cuda", u8=True)
        items = [tr.step(b0)]
        if graph:
            tr.capture(b1)
        items.append(tr.step(b1))
        # one more backward without the optimizer: the arena as the backward leaves it
        tr.forward_backward(b0)
        torch.cuda.synchronize()
        arena = tr.grad.clone()
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        ema = tr.ema_flat.clone()
        tr.graphs = None
        return torch.stack(items).cpu(), arena, sd, ema
    finally:
        K.LEVEL_STREAMS = old


@pytest.mark.parametrize("dtype,graph", [(torch.float32, False), (torch.float32, True), (torch.bfloat16, True)])
def test_levels_concurrent_bitwise_serial(dtype, graph):
    i0, a0, s0, e0 = _run(dtype, False, graph)
    i1, a1, s1, e1 = _run(dtype, True, graph)
    assert torch.equal(i0, i1), (i0, i1)
    bad = [k for k in s0 if not torch.equal(s0[k], s1[k])]
    assert not bad, bad[:10]
    assert torch.equal(e0, e1)
    assert torch.equal(a0, a1), float((a0 - a1).abs().max())


def test_levels_concurrent_eval_equal():
    from adrefine import kernels as K
    from adrefine.data.synthetic import images_u8
    m = _model(torch.bfloat16).eval()
    x = images_u8(4, 320, seed=9).cuda()
    outs = []
    for lv in (False, True):
        K.LEVEL_STREAMS = lv
        try:
            with torch.no_grad(), K.pack_scope(K.PackCache(cache_bn_coefs=True)):
                y = m(x)
            torch.cuda.synchronize()
            outs.append(y[0].clone())
        finally:
            K.LEVEL_STREAMS = False
    assert torch.equal(outs[0], outs[1])
