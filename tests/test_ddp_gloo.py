"""World-size-2 data parallelism on CPU (gloo): the host side of the DDP path — the staged forward/backward
(`tasks.route_layers` with cuts -> `ddp.staged_backward`) and the bucketed async all-reduce over the
stage-major gradient arena (`ddp.BucketReducer`) — on a small layered model routed exactly like the detector
(`m.f` / `m.i` / save list, a skip connection across both cuts).

Checks: (1) every rank's reduced arena equals the sum of both shards' gradients computed in one unstaged pass
(the reference's `loss *= world_size` + DDP average, trainer.py:387/273); (2) each bucket was launched only
after its stage's gradients were final (its value at launch time equals its final local value), in order
last stage -> first stage; (3) the staged backward leaves the same local gradients as an unstaged one."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from adrefine.engine.ddp import BucketReducer, stage_of, staged_backward
from adrefine.nn.tasks import route_layers

CUTS = (1, 2)


class Sum(nn.Module):
    def forward(self, xs):
        return xs[0] + xs[1]


def _toy(seed=0):
    torch.manual_seed(seed)
    spec = [(-1, nn.Linear(8, 16)), (-1, nn.Sequential(nn.Linear(16, 16), nn.Tanh())), (-1, nn.Linear(16, 16)),
            ([-1, 0], Sum()), (-1, nn.Linear(16, 4))]
    layers = []
    for i, (f, m) in enumerate(spec):
        m.i, m.f = i, f
        layers.append(m)
    save = [0]
    return nn.ModuleList(layers), save


def _params_by_stage(model):
    """(name, param) in arena order: stage-major, last stage first."""
    named = [(n, p) for n, p in model.named_parameters()]
    nst = len(CUTS) + 1
    return sorted(named, key=lambda e: nst - 1 - stage_of(int(e[0].split(".")[0]), CUTS))


def _arena(model):
    plist = _params_by_stage(model)
    n = sum(p.numel() for _, p in plist)
    arena = torch.zeros(n)
    ranges = [[None, None] for _ in range(len(CUTS) + 1)]
    off = 0
    for name, p in plist:
        p.grad = arena[off:off + p.numel()].view(p.shape)  # autograd accumulates in place into the arena
        s = stage_of(int(name.split(".")[0]), CUTS)
        ranges[s][0] = off if ranges[s][0] is None else ranges[s][0]
        off += p.numel()
        ranges[s][1] = off
    return arena, [tuple(r) for r in ranges]


def _loss(model, save, x, cuts):
    out, bounds = route_layers(list(model), save, x, [], 0, cuts)
    return (out ** 2).sum() * x.shape[0], bounds


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(3 + rank, 8, generator=g)  # ragged shards


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, save = _toy()
        # reference: both shards, unstaged, summed
        arena_ref, _ = _arena(model)
        for r in range(world):
            loss, _ = _loss(model, save, _data(r), ())
            loss.backward()
        expect = arena_ref.clone()
        # local staged backward of this rank's shard must equal the local unstaged one
        arena_u, _ = _arena(model)
        _loss(model, save, _data(rank), ())[0].backward()
        local_unstaged = arena_u.clone()
        arena, ranges = _arena(model)
        red = BucketReducer(arena, ranges, world)
        snaps = {}
        loss, bounds = _loss(model, save, _data(rank), CUTS)
        assert len(bounds) == len(CUTS)

        def after_stage(s):
            lo, hi = ranges[s]
            snaps[s] = arena[lo:hi].clone()  # local gradient at launch time
            red.launch(s)

        staged_backward(loss, bounds, lambda fn: fn(), after_stage)
        # the local arena before the reductions land is what each bucket held at launch
        order = red.wait()
        torch.testing.assert_close(arena, expect, rtol=1e-5, atol=1e-6)
        ok_final = True
        for s, (lo, hi) in enumerate(ranges):
            ok_final &= torch.allclose(snaps[s], local_unstaged[lo:hi], rtol=1e-5, atol=1e-6)
        q.put((rank, order, ok_final, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, False, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_staged_bucket_allreduce_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, order, ok_final, err in res:
        assert err is None, (rank, err)
        assert order == [2, 1, 0], order  # last stage first
        assert ok_final, f"rank {rank}: a bucket was launched before its stage's gradients were final"


def test_stage_layout_and_cut_leaves():
    """cut_live detaches exactly the tensors read across each cut (x and the saved skip y[0])."""
    model, save = _toy()
    x = _data(0)
    out, bounds = route_layers(list(model), save, x, [], 0, CUTS)
    assert [len(b) for b in bounds] == [2, 2]  # after L1: {y[0], x}; after L2: {y[0] leaf, x}
    for b in bounds:
        for t, leaf in b:
            assert leaf.is_leaf and leaf.requires_grad and leaf.data_ptr() == t.data_ptr()
    assert stage_of(0, CUTS) == 0 and stage_of(2, CUTS) == 1 and stage_of(4, CUTS) == 2


@pytest.mark.parametrize("bs,acc", [(16, 4), (64, 1), (512, 1), (8, 8)])
def test_trainer_setup_accumulate_and_decay(bs, acc):
    """accumulate = max(round(nbs / batch), 1) and the decay scaling (trainer.py:305-306) on the GLOBAL batch."""
    from adrefine.engine.trainer import Schedule
    s = Schedule(nbs=64, batch_size=bs)
    assert s.accumulate0 == acc
    assert abs(5e-4 * bs * acc / 64 - 5e-4 * bs * s.accumulate0 / 64) == 0
