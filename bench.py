"""Benchmark: YOLO-AD-Refine-n training step (fwd + TAL/DFL/CIoU+NWD loss + bwd + clip + SGD + EMA) on synthetic
640x640 batches, bs 64 per GPU (BASELINE.json configs[2] per GPU; configs[3] = 8 GPUs x 64 via DDP/RCCL).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--bs 64] [--img 640] [--dtype bf16|fp32]
  N>1: python bench.py --gpus N starts the N ranks itself (python -m torch.distributed.run ... as a child process);
       under an outside launcher (torch.distributed.run --nproc-per-node N ... bench.py --gpus N) it runs as a rank.
       WORLD_SIZE != N, or fewer than N visible GPUs: exit code 2 with the reason on stderr.
  python bench.py --infer [--infer-bs 32]   BASELINE.json configs[1]: batched inference (uint8 -> eval forward
                                            -> decode -> NMS) as its own JSON line

Prints ONE JSON line on rank 0 (value = images/s summed over all ranks; max-over-ranks timing). The training line
also carries a short configs[1] inference measurement under "inference" (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA (spec, no sparsity)
F32_MFMA_PEAK_TF = 157.3


def cpu_baseline(bs=2, img=640, budget_s=20.0):
    """The CPU oracle (oracle/adr_oracle.py, a pure-PyTorch restatement pinned to the reference) timed on the host
    cores: fwd + v8DetectionLoss + bwd for bs-image batches at img^2, until ~budget_s of work."""
    import torch
    import yaml
    sys.path.insert(1, str(ROOT / "oracle"))  # the oracle is the CPU baseline leg only
    import adr_oracle as O
    from recipe import recipe_state_dict, synthetic_images, synthetic_labels
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    d = yaml.safe_load(CFG.read_text())
    layers, save = O.parse(d, 3, None)
    import adrefine.nn.tasks as T  # only for the key/shape list (no GPU work)
    spec = [(k, tuple(v.shape)) for k, v in T.DetectionModel(str(CFG)).state_dict().items()]
    P = recipe_state_dict(spec)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k and not k.endswith("dfl.conv.weight"):
            v.requires_grad_(True)
    x = synthetic_images(bs, img, seed=0)
    lab = synthetic_labels(bs, 80, seed=1)
    n, t0 = 0, time.perf_counter()
    while True:
        preds = O.forward(P, layers, save, x, train=True)
        loss, _ = O.detection_loss(preds, lab["batch_idx"], lab["cls"], lab["bboxes"])
        loss.backward()
        for v in P.values():
            if v.grad is not None:
                v.grad = None
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * bs / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} steps x {bs} images @{img}^2 (fwd+loss+bwd, fp32, torch CPU {threads} threads)"}


def cpu_baseline_infer(bs=1, img=640, budget_s=8.0):
    """The CPU oracle's eval forward + decode (fp32, host cores) — the inference leg's baseline."""
    import torch
    import yaml
    sys.path.insert(1, str(ROOT / "oracle"))
    import adr_oracle as O
    from recipe import recipe_state_dict, synthetic_images
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    d = yaml.safe_load(CFG.read_text())
    layers, save = O.parse(d, 3, None)
    import adrefine.nn.tasks as T
    P = recipe_state_dict([(k, tuple(v.shape)) for k, v in T.DetectionModel(str(CFG)).state_dict().items()])
    x = synthetic_images(bs, img, seed=0)
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            y, _ = O.forward(P, layers, save, x, train=False)
            O.non_max_suppression(y, 0.25, 0.7)
            n += 1
            if time.perf_counter() - t0 > budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": round(n * bs / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} batches x {bs} images @{img}^2 (eval fwd + decode + NMS, fp32, torch CPU {threads} threads)"}


def infer_bench(model, bs, img, steps, warmup, dev, graph=True, roofline=False, conf=0.25, multi_label=False,
                nms_share=False):
    """BASELINE.json configs[1]: uint8 batch -> /255 in the stem -> eval forward (bf16) -> decode -> NMS
    (predictor settings conf 0.25, iou 0.7, max_det 300; or the validator's conf 0.001 + multi-label,
    engine/validator.py:98-99), one hipGraph per batch. Inputs resident in HBM; the timed region is `steps` graph
    replays between two synchronisations. Returns (images/s, ms/batch, roofline or None, detections per batch,
    NMS share or None): the share is the adr_nms launches' part of one eagerly timed batch (HIP events per
    launch)."""
    import torch
    import adrefine.kernels as K
    from adrefine.data.synthetic import images_u8
    from adrefine.engine.predictor import FusedPredictor
    was_training = model.training
    model.eval()
    x = images_u8(bs, img, seed=7).to(dev)
    pred = FusedPredictor(model, conf=conf, iou=0.7, max_det=300, multi_label=multi_label)
    for _ in range(warmup):
        pred.run_padded(x)
    if graph:
        pred.capture(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out, n = pred.run_padded(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    roof = share = None
    if roofline or nms_share:
        g, pred.graph = pred.graph, None
        K.timing_begin()
        pred.run_padded(x)
        recs = K.timing_end()
        if roofline:
            roof = K.roofline_report(recs, model.compute_dtype, HBM_PEAK_GBS,
                                     BF16_MFMA_PEAK_TF if model.compute_dtype == torch.bfloat16 else F32_MFMA_PEAK_TF)
        if nms_share:
            tot = sum(r[-1] for r in recs)
            nms = sum(r[-1] for r in recs if "nms" in str(r[0]).lower())
            share = {"nms_ms": round(1e3 * nms, 3), "batch_kernels_ms": round(1e3 * tot, 3),
                     "share": round(nms / tot, 4) if tot else None}
        pred.graph = g
    dets = int(n.sum())
    model.train(was_training)
    return bs * steps / dt, 1000 * dt / steps, roof, dets, share


def nms_bench(dev, bs=32, iters=20):
    """The NMS leg on a fixed, seeded head output (data/synthetic.head_output: bs 32 x 8400 anchors x 80 classes),
    so its work does not depend on the model state: adr_nms (one persistent launch) at the predictor's settings
    (conf 0.25, iou 0.7, single-label) and the validator's (conf 0.001, multi-label; engine/validator.py:98-99),
    max_det 300, max_nms 30000. HIP events on the launch stream around `iters` calls."""
    import torch
    from adrefine.data.synthetic import head_output
    from adrefine.utils.ops import check_counts, non_max_suppression_padded
    y = head_output(bs, seed=7).to(dev).contiguous()
    res = {"input": f"data/synthetic.head_output(bs={bs}, 8400 anchors, 80 classes, seed 7)"}
    for name, conf, multi in (("predict", 0.25, False), ("val", 0.001, True)):
        sc = y[:, 4:]
        cand = int((sc > conf).sum()) if multi else int((sc.amax(1) > conf).sum())
        for _ in range(3):
            out, n = non_max_suppression_padded(y, conf, 0.7, multi_label=multi)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            out, n = non_max_suppression_padded(y, conf, 0.7, multi_label=multi)
        e1.record()
        torch.cuda.synchronize()
        counts = n.tolist()
        check_counts(counts, dev)
        res[name] = {"conf": conf, "multi_label": multi, "candidates": cand, "detections_per_batch": sum(counts),
                     "us_per_call": round(1e3 * e0.elapsed_time(e1) / iters, 2), "calls": iters}
    return res


def pmc_traffic(symbol):
    """HBM bytes per launch of `symbol` from the committed PMC passes (profiles/pmc_traffic.json, written by
    scripts/pmc_traffic.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this same bench); (None, None)
    when the kernel was not covered. Matches the demangled name, or the unique entry the label is a prefix of."""
    import subprocess
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None
    doc = json.loads(f.read_text())
    name = symbol
    if symbol.startswith("_Z"):
        try:
            name = subprocess.run(["c++filt", symbol], capture_output=True, text=True, timeout=10).stdout.strip()
        except (OSError, subprocess.SubprocessError):
            return None, None
    rec = doc["kernels"].get(name)
    if rec is None:
        hits = [k for k in doc["kernels"] if k.replace("void ", "").startswith(name + "(")]
        m = re.match(r"adr::(\w+)<__bf16((?:, \d+)*)>$", name)
        if not hits and m:  # rocprofv3 leaves these templates mangled: _ZN3adr<len><name>IDF16b[Li<n>E...]E...
            base, nums = m.group(1), [int(v) for v in re.findall(r"\d+", m.group(2))]
            pre = f"_ZN3adr{len(base)}{base}IDF16b" + "".join(f"Li{v}E" for v in nums) + "E"
            hits = [k for k in doc["kernels"] if k.startswith(pre)]
        if not hits:  # rocprofv3 prints some instantiations as "adr::k<bool _Accum, int, E>(...)": the base name
            base = re.sub(r"^void ", "", name.split(" (")[0]).split("<")[0].split("(")[0]
            hits = [k for k in doc["kernels"] if k.startswith((f"void {base}<", f"{base}(", f"void {base}("))]
        if len(hits) != 1:
            return None, None
        rec = doc["kernels"][hits[0]]
    return rec["hbm_bytes_per_launch"], f"profiles/pmc_traffic.json ({rec['launches']} launches)"


# SURVEY.md §8d / BASELINE.md §3: per-image algorithmic work of the fwd+bwd step at n/640 (layer granularity)
NET_BYTES_PER_IMG = 210e6
NET_FLOPS_PER_IMG = 34.6e9


# the bf16 conv engine's fwd / dgrad kernels (incl. the Conv-BN-act XF variants)
_CONV_TAGS = ("_ZN3adr16conv_bf16", "_ZN3adr12conv3", "_ZN3adr12conv1", "_ZN3adr19conv_bf16_xf", "_ZN3adr15conv3_xf")


def conv_attainable(detail, hbm_gbs, mfma_tf):
    """Attainable-roofline fraction of the conv family (north_star: '>= 70 % CDNA4 bf16 MFMA roofline on the fused
    Conv-BN-SiLU backbone'): sum over conv fwd/dgrad launches of max(bytes / HBM peak, flops / MFMA peak)
    divided by their measured time."""
    ideal = meas = 0.0
    for tag, shape, nb, fl, t in detail:
        if nb is None or not tag.startswith(_CONV_TAGS):
            continue
        ideal += max(nb / (hbm_gbs * 1e9), fl / (mfma_tf * 1e12))
        meas += t
    return None if meas == 0 else {"launches_timed": sum(1 for d in detail if d[0].startswith(_CONV_TAGS)),
                                   "attainable_frac": round(ideal / meas, 4), "ms_total": round(1e3 * meas, 3)}


def stage_overhead(model, tr, batch, bs, steps=30):
    """configs[3] readiness on one GPU: the DDP step is staged (one graph per gradient bucket, the all-reduces
    between replays, engine/ddp.py); time that staged 1-GPU step against the unstaged one, back to back."""
    import torch
    from adrefine.engine.ddp import cuts_for_bucket
    from adrefine.engine.trainer import DDP_BUCKET_MB, FusedTrainer
    import socket

    import torch.distributed as dist
    cuts = cuts_for_bucket(model, DDP_BUCKET_MB)
    tr2 = FusedTrainer(model, batch_size=bs, world_size=1, stages=cuts)
    # the same staged step with the real RCCL bucket all-reduces between the stage-graph replays: a one-rank `nccl`
    # process group (the multi-GPU step's exact host / stream interleaving; the one-rank sum is the identity)
    tr3, rccl_err = None, None
    try:
        if not dist.is_initialized():
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                port = so.getsockname()[1]
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                    device_id=next(model.parameters()).device)
        tr3 = FusedTrainer(model, batch_size=bs, world_size=1, stages=cuts, collectives=True)
    except Exception as e:  # noqa: BLE001 - report, keep the line
        rccl_err = f"{type(e).__name__}: {e}"[:200]
    for t in (tr2, tr3):
        if t is None:
            continue
        for _ in range(3):
            t.step(batch)
        t.capture(batch)
        t.step(batch)

    def timed(t):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            t.step(batch)
        torch.cuda.synchronize()
        return 1000 * (time.perf_counter() - t0) / steps

    runs = {"un": [], "st": [], "rc": []}
    for _ in range(2):
        runs["un"].append(timed(tr))
        runs["st"].append(timed(tr2))
        if tr3 is not None:
            runs["rc"].append(timed(tr3))
    un, st = min(runs["un"]), min(runs["st"])
    rc = min(runs["rc"]) if runs["rc"] else None
    tr2.graphs = None
    if tr3 is not None:
        tr3.graphs = None
    return {"bucket_mb": DDP_BUCKET_MB, "cuts": list(cuts), "stages": len(cuts) + 1, "ms_per_step_unstaged": round(un, 3),
            "ms_per_step_staged": round(st, 3), "overhead": round(st / un - 1, 4), "steps": steps,
            "ms_per_step_staged_rccl": None if rc is None else round(rc, 3),
            "rccl_overhead_vs_staged": None if rc is None else round(rc / st - 1, 4),
            "rccl_overhead_vs_unstaged": None if rc is None else round(rc / un - 1, 4),
            "rccl": "one-rank nccl group, real all_reduce per bucket between stage-graph replays" if rccl_err is None
            else rccl_err}


def lscale_bench(dev, dtype, steps=10, warmup=3, bs=16, img=1280):
    """BASELINE.json configs[4] per GPU, as an object of the default line: the 701 yaml at l scale (depth/width
    1.0/1.0, nn/tasks.py:1050-1051), 1280^2, bs 16, the same captured train step (fwd + loss + bwd + SGD + EMA),
    `steps` timed replays after `warmup` eager steps + capture. MFMA fraction from BASELINE.md's 765.6 GFLOP
    forward per image (backward = 2x forward)."""
    import torch
    import yaml

    from adrefine.data.synthetic import train_batch
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    cfg = yaml.safe_load(CFG.read_text())
    cfg["scale"] = "l"
    torch.manual_seed(0)
    model = DetectionModel(cfg, compute_dtype=dtype).to(dev)
    tr = FusedTrainer(model, batch_size=bs, world_size=1)
    batch, _ = train_batch(bs, img, seed=11, device=dev, u8=True)
    for _ in range(warmup):
        tr.step(batch)
    tr.capture(batch)
    tr.step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        items = tr.step(batch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ips = bs * steps / dt
    peak = torch.cuda.max_memory_allocated(dev) / 2 ** 30
    finite = bool(torch.isfinite(items).all())
    tr.graphs, tr._sets = None, {}
    del tr, model
    torch.cuda.empty_cache()
    mfma_peak = BF16_MFMA_PEAK_TF if dtype == torch.bfloat16 else F32_MFMA_PEAK_TF
    return {"config": f"BASELINE configs[4] per GPU: yolo11-701-YOLO-AD-Refine.yaml (l) train step bs={bs} "
                      f"{img}x{img}, hipGraph, {steps} timed steps after {warmup} warm-up + capture",
            "value": round(ips, 2), "unit": "images/s", "ms_per_step": round(1000 * dt / steps, 3),
            "flops_per_img": 3 * 765.6e9, "mfma_frac": round(ips * 3 * 765.6e9 / (mfma_peak * 1e12), 4),
            "peak_hbm_gib": round(peak, 2), "loss_finite": finite, "dtype": str(dtype).split(".")[-1],
            "fp8": "not used: the e4m3 forward-conv engine (--conv-fp8) is not faster than bf16 at this config "
                   "(DESIGN.md §9)"}


def step_traffic():
    """Whole-step HBM traffic per image from profiles/step_traffic.json (scripts/step_traffic.py: PMC bytes per
    launch x launches per replayed step, per kernel); None when absent."""
    f = ROOT / "profiles" / "step_traffic.json"
    if not f.exists():
        return None
    d = json.loads(f.read_text())
    return {"traffic_bytes_per_img": d["traffic_bytes_per_img"], "traffic_over_alg": d["traffic_over_alg"],
            "coverage_of_kernel_time": d["coverage"], "source": "profiles/step_traffic.json (" + d["source"] + ")"}


def augment_bench(bs, img, dev, reps=5):
    """The training augmentation chain (data/augment.py v8_transforms, default hyp) on a synthetic dataset: host side
    (draws, labels, plans) per batch and the fused GPU render (adr_augment_u8) per batch, HIP events on its stream."""
    import random
    from types import SimpleNamespace

    import numpy as np
    import torch

    from adrefine.data.augment import Format, collate_fn, render, v8_transforms
    from adrefine.data.synthetic import AugSourceDataset

    hyp = SimpleNamespace(mosaic=1.0, degrees=0.0, translate=0.1, scale=0.5, shear=0.0, perspective=0.0, flipud=0.0,
                          fliplr=0.5, hsv_h=0.015, hsv_s=0.7, hsv_v=0.4, mixup=0.0, copy_paste=0.0,
                          copy_paste_mode="flip", bgr=0.0)
    ds = AugSourceDataset(2 * bs, img, seed=4)
    T = v8_transforms(ds, img, hyp)
    T.append(Format(bbox_format="xywh", normalize=True, batch_idx=True, bgr=0.0))
    random.seed(0)
    np.random.seed(0)
    host, kern = [], []
    out = torch.empty(bs, 3, img, img, dtype=torch.uint8, device=dev)
    for r in range(reps + 1):
        t0 = time.perf_counter()
        samples = [T(ds.get_image_and_label(i % len(ds))) for i in range(bs)]
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        plans = [smp["img"] for smp in samples]
        render(plans, dev, out=out)  # uploads the sources, then the kernel
        torch.cuda.synchronize()
        e0.record()
        render(plans, dev, out=out)
        e1.record()
        torch.cuda.synchronize()
        if r:
            host.append(t1 - t0)
            kern.append(e0.elapsed_time(e1))
    _ = collate_fn(samples, dev)
    host.sort()
    kern.sort()
    return {"pipeline": "Mosaic(4) -> RandomPerspective(warpAffine) -> RandomHSV -> RandomFlip -> Format, default hyp; "
                        "pixels: one adr_augment_u8 launch per batch (render incl. the H2D upload of the sources)",
            "bs": bs, "img": img, "host_ms_per_batch": round(1000 * host[len(host) // 2], 2),
            "render_ms_per_batch": round(kern[len(kern) // 2], 3),
            "render_images_per_s": round(bs / (kern[len(kern) // 2] / 1000), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # 100 timed steps after 20 warm-up, median
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--img", type=int, default=640)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel from Python (no hipGraph replay)")
    ap.add_argument("--roofline-steps", type=int, default=2)
    ap.add_argument("--stage-check", type=int, default=1, help="time the DDP-staged step on 1 GPU (configs[3])")
    ap.add_argument("--float-images", action="store_true", help="feed pre-normalised fp32 images instead of uint8")
    ap.add_argument("--infer", action="store_true", help="measure BASELINE.json configs[1] (batched inference) only")
    ap.add_argument("--infer-bs", type=int, default=32)
    ap.add_argument("--infer-steps", type=int, default=20)
    ap.add_argument("--scale", default="n", choices=["n", "s", "m", "l", "x"],
                    help="model scale of the 701 yaml (configs[4] = l at 1280^2, bs 16/GPU)")
    ap.add_argument("--augment-bench", type=int, default=1, help="time the GPU training augmentation chain")
    ap.add_argument("--lscale-steps", type=int, default=10,
                    help="timed steps of the configs[4] l/1280/bs16 object in the default line (0: skip)")
    ap.add_argument("--conv-fp8", action="store_true",
                    help="forward convs on the fp8 (e4m3) MFMA engine (configs[4]'s fp8 conv path; backward bf16)")
    ap.add_argument("--ddp-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend of the N-rank run (nccl = RCCL over xGMI; gloo for tests)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="tests only (with --ddp-backend gloo): every rank on GPU rank %% visible, so the N-rank "
                         "launch path runs on a one-GPU box")
    args = ap.parse_args()
    if args.share_gpu and args.ddp_backend != "gloo":
        print("bench.py: --share-gpu needs --ddp-backend gloo (RCCL refuses two ranks on one GPU)", file=sys.stderr)
        sys.exit(2)
    # --gpus N: validate against the environment and start the N ranks ourselves when no launcher did, all before
    # any GPU call (a child process, never exec; trainer.py:184-204 / utils/dist.py:56-66)
    from adrefine.engine.ddp import LaunchError, check_world, launch_ranks
    try:
        mode = check_world(args.gpus, share_gpu=args.share_gpu)
    except LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "launch":
        sys.exit(launch_ranks(args.gpus, Path(__file__).resolve(), sys.argv[1:]))
    if args.scale != "n":  # configs[4]: its own line; the n/640 baselines (CPU, inference) do not apply
        args.no_cpu_baseline, args.infer_steps = True, 0

    import torch
    import torch.distributed as dist

    from adrefine.engine.ddp import setup_ddp
    rank, local, world, dev = setup_ddp(backend=args.ddp_backend, share_gpu=args.share_gpu)
    import adrefine.kernels as K
    K.CONV_FP8 = K.CONV_FP8 or args.conv_fp8
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.data.synthetic import train_batch
    from adrefine.nn.tasks import DetectionModel

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    if args.scale == "n":
        model = DetectionModel(str(CFG), compute_dtype=dtype).to(dev)
    else:
        import yaml
        cfg = yaml.safe_load(CFG.read_text())
        cfg["scale"] = args.scale
        model = DetectionModel(cfg, compute_dtype=dtype).to(dev)
    if args.infer:
        ips, ms, roof, dets, _ = infer_bench(model, args.infer_bs, args.img, args.steps, args.warmup, dev,
                                             graph=not args.no_graph, roofline=True)
        if roof is not None:
            roof["traffic"], roof["traffic_source"] = None, None
        if rank == 0:
            cpu = None if args.no_cpu_baseline else cpu_baseline_infer()
            print(json.dumps({
                "metric": "images/sec inference (640x640) bs32, YOLO-AD-Refine-n, 1 GPU",
                "value": round(world * ips, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (uint8 images)",
                "config": {"workload": f"yolo11-701-YOLO-AD-Refine.yaml (n) inference bs={args.infer_bs} "
                                       f"{args.img}x{args.img}: uint8 -> eval fwd -> DFL decode -> NMS(conf 0.25, "
                                       f"iou 0.7, max_det 300)", "global_batch": world * args.infer_bs,
                           "img": args.img, "parallelism": f"replicas{world}"},
                "roofline": roof, "cpu_baseline": cpu, "detections_per_batch": dets,
                "hipgraph": not args.no_graph}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if world > 1:  # same initial weights on every rank (DDP broadcasts rank 0's parameters at construction)
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    # the reference's batch_size is the GLOBAL batch (trainer.py:290, 305-306): accumulate and weight decay
    tr = FusedTrainer(model, batch_size=world * args.bs, world_size=world)
    # rank's shard of the stream, as the dataloader yields it: uint8 images (preprocess_batch's /255 runs inside the
    # step, fused into the stem kernels) + COCO-shape labels
    batch, _ = train_batch(args.bs, args.img, seed=1000 * rank, device=dev, u8=not args.float_images)

    for _ in range(args.warmup):
        tr.step(batch)
    if not args.no_graph:
        tr.capture(batch)  # fwd+loss+bwd and the optimizer tail as two hipGraphs (all-reduce between them)
        tr.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    for k in range(args.steps):
        items = tr.step(batch)
        ev[k + 1].record()  # per-step boundaries on the step's stream (median / p90; the value uses the wall clock)
    t_host = time.perf_counter() - t0  # host-side enqueue time (launch-bound if close to the step time)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # per-kernel durations for the roofline: HIP events on the launch stream around every conv-GEMM launch of
    # the same step, run eagerly right after the timed replays (a graph replay cannot be split per kernel)
    peak_gib = torch.cuda.max_memory_allocated(dev) / 2 ** 30  # caching-allocator peak over warmup + capture + steps
    graphs, tr.graphs = tr.graphs, None
    K.timing_begin()
    for _ in range(args.roofline_steps):
        tr.step(batch)
    ktimes = K.timing_end()
    tr.graphs = graphs
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    ips = world * args.bs * args.steps / dt
    per = sorted(ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps))
    step_stats = {"median": round(per[len(per) // 2], 3), "p10": round(per[len(per) // 10], 3),
                  "p90": round(per[(9 * len(per)) // 10], 3), "min": round(per[0], 3)}
    if rank == 0:
        finite = bool(torch.isfinite(items).all())
        mfma_peak = BF16_MFMA_PEAK_TF if dtype == torch.bfloat16 else F32_MFMA_PEAK_TF
        roof = K.roofline_report(ktimes, dtype, HBM_PEAK_GBS, mfma_peak)
        if roof is not None:
            roof["traffic"], roof["traffic_source"] = pmc_traffic(roof["kernel"])
            if args.scale == "n" and args.img == 640:
                roof["network"] = {"bytes_per_img": NET_BYTES_PER_IMG, "flops_per_img": NET_FLOPS_PER_IMG,
                                   "hbm_frac": round(ips * NET_BYTES_PER_IMG / (HBM_PEAK_GBS * 1e9), 4),
                                   "mfma_frac": round(ips * NET_FLOPS_PER_IMG / (mfma_peak * 1e12), 4)}
                st = step_traffic()
                if st is not None and args.bs == 64:
                    roof["network"].update(st)
                    roof["network"]["traffic_gbs_at_this_step_rate"] = round(
                        ips * st["traffic_bytes_per_img"] / 1e9, 1)
            elif args.scale == "l" and args.img == 1280:  # 765.6 GFLOP fwd per image, bwd = 2x fwd
                roof["network"] = {"flops_per_img": 3 * 765.6e9,
                                   "mfma_frac": round(ips * 3 * 765.6e9 / (mfma_peak * 1e12), 4)}
            roof["conv_family"] = conv_attainable(K.timing_detail(), HBM_PEAK_GBS, mfma_peak)
        staging = None
        if world == 1 and args.stage_check and not args.no_graph:
            staging = stage_overhead(model, tr, batch, args.bs)
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(budget_s=args.cpu_budget)
        infer = nms = None
        if world == 1 and args.infer_steps > 0:  # configs[1] alongside the headline line
            # on a freshly initialised model (seed 0), not on the weights the timed train steps left, so the
            # inference leg's NMS work does not depend on how many steps ran before it
            torch.manual_seed(0)
            imodel = DetectionModel(str(CFG), compute_dtype=dtype).to(dev)
            i_ips, i_ms, _, dets, _ = infer_bench(imodel, args.infer_bs, args.img, args.infer_steps, 2, dev,
                                                  graph=not args.no_graph)
            # the validator's NMS settings (conf 0.001, multi-label: engine/validator.py:98-99) give NMS real work on
            # random-recipe logits (conf 0.25 leaves nothing to sort or suppress)
            v_ips, v_ms, _, v_dets, v_share = infer_bench(imodel, args.infer_bs, args.img, args.infer_steps, 2, dev,
                                                          graph=not args.no_graph, conf=0.001, multi_label=True,
                                                          nms_share=True)
            del imodel
            nms = nms_bench(dev, args.infer_bs)
            infer = {"metric": "images/sec inference (640x640) bs32, 1 GPU", "value": round(i_ips, 2),
                     "ms_per_batch": round(i_ms, 3), "bs": args.infer_bs, "steps": args.infer_steps,
                     "pipeline": "uint8 -> eval fwd (bf16) -> DFL decode -> NMS(0.25, 0.7, 300), one hipGraph",
                     "detections_per_batch": dets,
                     "val_nms": {"pipeline": "same, NMS(conf 0.001, iou 0.7, multi-label, max_det 300)",
                                 "value": round(v_ips, 2), "ms_per_batch": round(v_ms, 3),
                                 "detections_per_batch": v_dets, "nms_kernels": v_share}}
        out = {
            "metric": ("images/sec whole-node (640x640) fwd+bwd, YOLO-AD-Refine-n at 1/2/4/8 GPU" if args.scale == "n"
                       else f"images/sec whole-node ({args.img}x{args.img}) fwd+bwd, YOLO-AD-Refine-{args.scale}"),
            "value": round(ips, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype + ("+fp8-fwd-conv" if K.CONV_FP8 else ""),
            "data": "synthetic (uint8 images + COCO-shape labels)" if not args.float_images else "synthetic (fp32 images)",
            "config": {"workload": f"yolo11-701-YOLO-AD-Refine.yaml ({args.scale}) train step bs={args.bs}/GPU "
                                   f"{args.img}x{args.img}, synthetic COCO-shape labels, TAL+DFL+CIoU/NWD loss, "
                                   f"SGD+EMA", "global_batch": world * args.bs, "img": args.img,
                       "parallelism": f"dp{world}",
                       "ddp": None if world == 1 else {"backend": args.ddp_backend, "launched_by": (
                           "bench.py --gpus (child torch.distributed.run)" if os.environ.get("ADR_SELF_LAUNCHED")
                           else "outside launcher"), "shared_gpu": args.share_gpu},
                       "nms": "not in the train step (measured in the inference leg at validator settings)"},
            "roofline": roof, "cpu_baseline": cpu, "loss_finite": finite,
            "ms_per_step_events": step_stats, "ddp_staging": staging,
            "host_enqueue_ms_per_step": round(1000 * t_host / args.steps, 3), "hipgraph": not args.no_graph,
            "inference": infer, "nms": nms, "peak_hbm_gib": round(peak_gib, 2),
            "augment": (augment_bench(args.bs, args.img, dev) if world == 1 and args.augment_bench and
                        args.scale == "n" else None),
        }
        if world == 1 and args.scale == "n" and args.lscale_steps > 0 and not args.no_graph:
            graphs, tr.graphs, tr._sets = tr.graphs, None, {}  # free the n step's graph pool first
            del graphs
            torch.cuda.empty_cache()
            out["lscale"] = lscale_bench(dev, dtype, steps=args.lscale_steps)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
