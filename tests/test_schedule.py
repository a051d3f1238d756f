"""FusedTrainer's per-batch schedule (engine/trainer.py Schedule) vs the reference's own loop structure
(engine/trainer.py:209-215 LambdaLR, :305 accumulate, :330 nw, :346-398 epoch/batch loop with warm-up
interpolation and the `ni - last_opt_step >= accumulate` optimizer-step rule), replayed here with a real
torch.optim.SGD whose param_groups are ordered (g2 bias, g0 decay, g1 norm) as build_optimizer :798-808 does."""
import math

import numpy as np
import pytest
import torch

from adrefine.engine.trainer import Schedule


def _reference_trace(lr0, lrf, momentum, nbs, batch, epochs, nb, warmup_epochs, wb_lr, w_mom, cos_lr):
    ps = [torch.nn.Parameter(torch.zeros(1)) for _ in range(3)]
    opt = torch.optim.SGD([ps[0]], lr=lr0, momentum=momentum, nesterov=True)  # g2 (bias)
    opt.add_param_group({"params": [ps[1]], "weight_decay": 1e-3})  # g0
    opt.add_param_group({"params": [ps[2]], "weight_decay": 0.0})  # g1
    if cos_lr:
        lf = lambda x: ((1 - math.cos(x * math.pi / epochs)) / 2) * (lrf - 1) + 1  # noqa: E731
    else:
        lf = lambda x: max(1 - x / epochs, 0) * (1.0 - lrf) + lrf  # noqa: E731
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lf)
    accumulate = max(round(nbs / batch), 1)
    nw = max(round(warmup_epochs * nb), 100) if warmup_epochs > 0 else -1
    last_opt_step = -1
    sched.last_epoch = -1
    trace = []
    for epoch in range(epochs):
        sched.step()
        for i in range(nb):
            ni = i + nb * epoch
            if ni <= nw:
                xi = [0, nw]
                accumulate = max(1, int(np.interp(ni, xi, [1, nbs / batch]).round()))
                for j, x in enumerate(opt.param_groups):
                    x["lr"] = np.interp(ni, xi, [wb_lr if j == 0 else 0.0, x["initial_lr"] * lf(epoch)])
                    if "momentum" in x:
                        x["momentum"] = np.interp(ni, xi, [w_mom, momentum])
            stepped = ni - last_opt_step >= accumulate
            if stepped:
                last_opt_step = ni
            g = opt.param_groups
            trace.append(([float(g[1]["lr"]), float(g[2]["lr"]), float(g[0]["lr"])], float(g[0]["momentum"]),
                          stepped))
    return trace


@pytest.mark.parametrize("batch,nb,epochs,warm,cos", [(16, 40, 6, 3.0, False), (64, 30, 5, 3.0, True),
                                                     (8, 150, 2, 0.5, False), (16, 20, 3, 0.0, False)])
def test_schedule_matches_reference_loop(batch, nb, epochs, warm, cos):
    ref = _reference_trace(0.01, 0.01, 0.937, 64, batch, epochs, nb, warm, 0.1, 0.8, cos)
    s = Schedule(lr0=0.01, lrf=0.01, momentum=0.937, nbs=64, batch_size=batch, epochs=epochs, nb=nb,
                 warmup_epochs=warm, warmup_bias_lr=0.1, warmup_momentum=0.8, cos_lr=cos)
    last = -1
    nsteps = 0
    for ni, (lrs, mom, stepped) in enumerate(ref):
        mlrs, mmom, acc = s.at(ni)
        assert np.allclose(mlrs, lrs, rtol=1e-12, atol=1e-15), (ni, mlrs, lrs)
        assert abs(mmom - mom) < 1e-12, (ni, mmom, mom)
        mine = ni - last >= acc
        assert mine == stepped, (ni, acc)
        if mine:
            last = ni
            nsteps += 1
    assert nsteps < len(ref) or batch >= 64


def test_constant_schedule_without_nb():
    s = Schedule(lr0=0.02, momentum=0.9, nbs=64, batch_size=16)
    assert s.at(0) == ([0.02] * 3, 0.9, 4) and s.at(1000) == ([0.02] * 3, 0.9, 4)
