"""The RCCL code path of the DDP step on the one GPU of the box (configs[3]'s collective, engine/ddp.py): a child
process initialises torch.distributed with backend `nccl` (RCCL) and world_size 1 before any other GPU work, then
FusedTrainer(collectives=True) issues real async all_reduce(SUM) calls on every gradient bucket between the replays
of its captured stage graphs — the interleaving the reference's DDP hooks produce during backward
(engine/trainer.py:273, 387, 393). A one-rank sum is the identity, so the step must be BITWISE equal to the same
staged step without collectives: parameters, EMA and loss items after each of two graph-replayed steps. The stage
graphs are captured while an async all_reduce is still in flight (the condition under which a global-mode capture
aborted the r04t bench: the RCCL watchdog's event query during capture); capture must complete and the bitwise
checks hold."""
import json
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_staged_step_bitwise():
    cmd = [sys.executable, str(ROOT / "tests" / "rccl_step.py"), str(_free_port()), "320", "8", "10"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(line[-1][7:])
    print(res)
    assert res["backend"] == "nccl" and res["world_size"] == 1 and len(res["cuts"]) >= 3
    assert res["pending_at_capture"], res  # the capture ran while the watchdog had an in-flight collective to poll
    for st in res["steps"]:
        assert st["loss_finite"] and st["params_equal"] and st["ema_equal"] and st["items_equal"], res
