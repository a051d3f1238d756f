"""`bench.py --gpus N` / engine/ddp.py process launch (CPU): the command the self-launch builds, the checks that
refuse a request the node cannot run, and the per-rank group setup with gloo at world size 2. Reference:
engine/trainer.py:184-204 (re-run as a DDP subprocess when world_size > 1 and LOCAL_RANK is unset), :217-228
(_setup_ddp), utils/dist.py:56-66 (generate_ddp_command)."""
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT
from adrefine.engine.ddp import LaunchError, check_world, generate_ddp_command, setup_ddp


def test_generate_ddp_command():
    cmd = generate_ddp_command(8, "/x/bench.py", ["--gpus", "8", "--steps", "5"], port=29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "8", "--steps", "5"]
    p = generate_ddp_command(2, "b.py", [])
    port = int(p[p.index("--master-port") + 1])
    assert 0 < port < 65536


def test_check_world_modes():
    assert check_world(1, env={}) == "single"
    assert check_world(8, env={}, visible=8) == "launch"
    assert check_world(8, env={"WORLD_SIZE": "8"}) == "rank"
    assert check_world(1, env={"WORLD_SIZE": "1"}) == "single"
    assert check_world(2, env={}, visible=1, share_gpu=True) == "launch"


@pytest.mark.parametrize("gpus,env,visible,msg", [
    (8, {"WORLD_SIZE": "4"}, 8, "WORLD_SIZE=4"),
    (1, {"WORLD_SIZE": "8"}, 8, "WORLD_SIZE=8"),
    (8, {}, 1, "1 GPU(s) are visible"),
    (2, {}, 0, "0 GPU(s) are visible"),
    (0, {}, 8, "must be >= 1"),
])
def test_check_world_refuses(gpus, env, visible, msg):
    with pytest.raises(LaunchError, match=msg.replace("(", r"\(").replace(")", r"\)")):
        check_world(gpus, env=env, visible=visible)


def _bench(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, env=env, cwd=str(ROOT))


def test_bench_refuses_mismatch_and_missing_gpus():
    """Exit code 2 and the reason on stderr, before any GPU work: WORLD_SIZE != --gpus; more ranks than visible
    GPUs (none here); --share-gpu without gloo."""
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "4"})
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr and "--gpus 2" in r.stderr, r.stderr[-2000:]
    r = _bench(["--gpus", "2"], {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 2 and "GPU(s) are visible" in r.stderr, r.stderr[-2000:]
    r = _bench(["--gpus", "2", "--share-gpu"], {})
    assert r.returncode == 2 and "gloo" in r.stderr, r.stderr[-2000:]


def _setup_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch
    import torch.distributed as dist
    r, lr, w, dev = setup_ddp(backend="gloo", timeout_s=60)
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    q.put((r, lr, w, str(dev), float(t), dist.get_backend()))
    dist.destroy_process_group()


def test_setup_ddp_gloo_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_setup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert [o[0] for o in out] == [0, 1] and all(o[2] == 2 and o[4] == 3.0 and o[5] == "gloo" for o in out)
    assert all(o[3] == "cpu" for o in out)


def test_setup_ddp_nccl_without_gpu_raises():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    os.environ.pop("WORLD_SIZE", None)
    with pytest.raises(LaunchError):
        setup_ddp(backend="nccl")
