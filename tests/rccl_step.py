"""Child process of tests/test_gpu_rccl.py (and bench.py's ddp_staging RCCL leg reuses the same idea): initialises
the `nccl` (RCCL) backend with world_size 1 BEFORE any other GPU work, then runs the DDP-staged training step with
real bucket all-reduces between the captured stage graphs (FusedTrainer(collectives=True)) next to the same staged
step without collectives, and prints one JSON line: bitwise equality of parameters / EMA / loss items after each
step, and per-step times. The collective trainer's graphs are captured while an async all_reduce is still pending
(pending_at_capture). usage: python tests/rccl_step.py <port> <img> <bs> <steps>"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    port, img, bs, steps = (int(v) for v in sys.argv[1:5])
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    from adrefine.data.synthetic import train_batch
    from adrefine.engine.ddp import cuts_for_bucket
    from adrefine.engine.trainer import DDP_BUCKET_MB, FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    cfg = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
    trainers = []
    for coll in (True, False):
        torch.manual_seed(0)
        m = DetectionModel(str(cfg), compute_dtype=torch.bfloat16).to(dev)
        cuts = cuts_for_bucket(m, min(DDP_BUCKET_MB, 4.0))  # four stages: every inter-stage path exercised
        trainers.append(FusedTrainer(m, batch_size=bs, world_size=1, stages=cuts, collectives=coll))
    batches = [train_batch(bs, img, seed=s, device=dev, u8=True)[0] for s in (11, 12, 13, 14)]
    res = {"cuts": list(trainers[0].cuts), "backend": dist.get_backend(), "world_size": dist.get_world_size(),
           "steps": []}
    for tr in trainers:
        tr.step(batches[0])
        tr.step(batches[1])
        if tr.collectives:
            # the r04t abort's condition: the graphs are captured while an async all_reduce is still in flight, so
            # the RCCL watchdog thread queries its work event DURING the capture (global capture mode aborts there;
            # the trainer captures in thread_local mode). A queued spin kernel keeps the collective pending.
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.cuda._sleep(1 << 20)
            e1.record()
            torch.cuda.synchronize()
            cycles = int((1 << 20) * 1500.0 / max(e0.elapsed_time(e1), 1e-3))  # ~1.5 s of spinning
            torch.cuda._sleep(cycles)
            work = dist.all_reduce(torch.ones(1 << 20, device=dev), async_op=True)
            res["pending_at_capture"] = not work.is_completed()
            tr.capture(batches[2])
            res["pending_after_capture"] = not work.is_completed()
            work.wait()
        else:
            tr.capture(batches[2])
    for b in batches[2:]:
        items = [tr.step(b) for tr in trainers]
        torch.cuda.synchronize()
        eq_p = all(torch.equal(p, q) for p, q in zip(trainers[0].model.parameters(), trainers[1].model.parameters()))
        eq_e = torch.equal(trainers[0].ema_flat, trainers[1].ema_flat)
        res["steps"].append({"params_equal": eq_p, "ema_equal": eq_e, "items_equal": torch.equal(*items),
                             "loss_finite": bool(torch.isfinite(items[0]).all())})
    times = {}
    for rep in range(2):
        for tr, name in zip(trainers, ("rccl", "none")):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                tr.step(batches[2])
            torch.cuda.synchronize()
            ms = 1000 * (time.perf_counter() - t0) / steps
            times[name] = min(times.get(name, 1e9), ms)
    res["ms_per_step_staged_rccl"] = round(times["rccl"], 3)
    res["ms_per_step_staged"] = round(times["none"], 3)
    res["rccl_overhead"] = round(times["rccl"] / times["none"] - 1, 4)
    dist.destroy_process_group()
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
