"""`bench.py --gpus N` on the one-GPU box (configs[3]'s launch path; trainer.py:184-204, utils/dist.py:56-66):
(1) --gpus 2 with one visible GPU exits 2 with the reason, before any GPU work; (2) the self-launch really runs
N ranks: --gpus 2 with gloo ranks sharing the one GPU (RCCL refuses two ranks on one device) starts a child
torch.distributed.run, both ranks run the staged, captured DDP step (bucket all-reduces between the stage-graph
replays) and rank 0 prints one JSON line with n_gpus 2 and the global batch."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(args, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


def test_bench_gpus2_on_one_gpu_refused():
    import torch
    n = torch.cuda.device_count()
    if n >= 2:
        pytest.skip(f"{n} GPUs visible")
    r = _bench(["--gpus", "2"], 120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert f"{n} GPU(s) are visible" in r.stderr


@pytest.mark.timeout(420)
def test_bench_gpus2_self_launch_gloo_shared_gpu():
    r = _bench(["--gpus", "2", "--ddp-backend", "gloo", "--share-gpu", "--steps", "3", "--warmup", "2", "--bs", "4",
                "--img", "320", "--no-cpu-baseline", "--stage-check", "0", "--augment-bench", "0",
                "--infer-steps", "0", "--roofline-steps", "1"], 400)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "DDP: launching" in r.stderr and "torch.distributed.run" in r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["ddp"]["backend"] == "gloo" and out["config"]["ddp"]["launched_by"].startswith("bench.py")
    assert out["loss_finite"] and out["value"] > 0
