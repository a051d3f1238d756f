"""Data-parallel plumbing of the training step: staged backward + bucketed gradient all-reduce.

The reference wraps the model in DistributedDataParallel (engine/trainer.py:273) whose autograd hooks all-reduce
gradient buckets while `scaler.scale(loss).backward()` (:393) is still running, so communication of the late
layers' gradients overlaps the backward of the early layers. This build keeps every parameter gradient in ONE
flat fp32 arena written by the kernels themselves (no per-parameter hooks), so it gets the same overlap a
different way:

* the layer list is cut into stages (`cuts` = layer indices after which a stage ends; by default where the
  gradient filled from the last layer reaches ~8 MB: after L10, two stages — trainer.DDP_BUCKET_MB) and the tensors that cross a cut are detached into fresh leaves during the forward
  (`cut_live`), so the backward runs stage by stage, last stage first (`staged_backward`);
* the arena is laid out stage-major, last stage first (`stage_of`, FusedTrainer), so when a stage's backward
  (and its batched WGRAD reductions) is done, its parameters' gradients form one contiguous bucket;
* `BucketReducer.launch(k)` starts an async all-reduce(SUM) of that bucket (RCCL over xGMI with backend "nccl",
  or gloo) while the next stage's backward is enqueued behind it on the compute stream.

With hipGraph replay (FusedTrainer.capture) every stage's backward is its own graph, and the collectives are
launched eagerly between the replays — the graphs themselves hold no collective.

Summing the per-rank gradients equals the reference's `loss *= world_size` (trainer.py:387) followed by DDP's
gradient average. BatchNorm statistics stay per rank as in the reference (no SyncBatchNorm). DDP also
broadcasts rank 0's buffers every forward (broadcast_buffers=True); batch-statistics BN never reads them in
training, rank 0's running statistics are rank 0's own update chain either way, and only rank 0's model/EMA is
saved or validated (trainer.py:436-444) — so skipping that broadcast changes nothing observable.
"""
from __future__ import annotations

import os
import re
import socket
import subprocess
import sys
from datetime import timedelta

import torch

_LAYER = re.compile(r"^model\.(\d+)\.")


def layer_of(name: str) -> int:
    """Layer index of a DetectionModel parameter / buffer name ('model.<i>.…'); -1 when it has none."""
    m = _LAYER.match(name)
    return int(m.group(1)) if m else -1


def stage_of(layer: int, cuts) -> int:
    """Stage index of a layer: stage s holds the layers after cuts[s-1] up to and including cuts[s]."""
    s = 0
    for c in sorted(cuts):
        if layer > c:
            s += 1
    return s


def cuts_for_bucket(model, bucket_mb=4.0):
    """Stage cuts whose parameter-gradient buckets hold about `bucket_mb` MB of fp32 gradients each, filled from the
    last layer down (the backward's order; the reference's DDP bucket_cap is 25 MB, trainer.py:273 — on
    point-to-point xGMI links a few MB per bucket starts the first all-reduce early without per-bucket latency
    dominating). A layer is never split: a single layer larger than the bucket is a bucket of its own. Returns
    the sorted layer indices after which a stage ends."""
    per = {}
    for name, p in model.named_parameters():
        li = layer_of(name)
        if li >= 0:
            per[li] = per.get(li, 0) + 4 * p.numel()
    if not per:
        return ()
    cap = bucket_mb * 2 ** 20
    cuts, acc = [], 0
    for li in range(max(per), 0, -1):
        acc += per.get(li, 0)
        if acc >= cap:
            cuts.append(li - 1)  # layers li.. form the bucket; the stage below ends at li - 1
            acc = 0
    return tuple(sorted(c for c in cuts if c >= 0))


def detach_leaf(t):
    """A leaf view of t (same storage and strides) that collects the gradient flowing back to t."""
    if not torch.is_tensor(t) or not t.requires_grad:
        return t
    leaf = t.detach()
    leaf.requires_grad_(True)
    return leaf


def cut_live(x, y, layers, i, bounds):
    """At the end of layer i: replace every tensor that a later layer reads (y[j] for j <= i in a later `f`, and
    x when layer i+1 reads -1) by a detached leaf, and record (tensor, leaf) pairs in `bounds`. Returns x."""
    later = layers[i + 1:]
    need = set()
    for m in later:
        for j in ([m.f] if isinstance(m.f, int) else m.f):
            if j != -1 and j <= i:
                need.add(j)
    pairs = []
    seen = {}
    for j in sorted(need):
        t = y[j]
        if t is None:
            raise RuntimeError(f"stage cut after layer {i}: layer {j}'s output is read later but not saved")
        if id(t) not in seen:
            seen[id(t)] = detach_leaf(t)
            pairs.append((t, seen[id(t)]))
        y[j] = seen[id(t)]
    if later and (later[0].f == -1 or (not isinstance(later[0].f, int) and -1 in later[0].f)):
        if id(x) not in seen:
            seen[id(x)] = detach_leaf(x)
            pairs.append((x, seen[id(x)]))
        x = seen[id(x)]
    bounds.append([(t, leaf) for t, leaf in pairs if leaf is not t])
    return x


def staged_backward(loss, bounds, run, after_stage):
    """Backward of a forward that was cut into len(bounds)+1 stages: the last stage from `loss`, then every
    earlier stage from the gradients its leaves collected. `run(fn)` wraps each stage's backward (the trainer
    passes its WGRAD deferral scope, so a stage's gradients are complete when it returns); `after_stage(s)` is
    called once stage s's parameter gradients are final."""
    S = len(bounds) + 1
    run(lambda: loss.backward())
    after_stage(S - 1)
    for k in range(S - 2, -1, -1):
        ts, gs = [], []
        for t, leaf in bounds[k]:
            if leaf.grad is not None:
                ts.append(t)
                gs.append(leaf.grad)
        if ts:
            run(lambda: torch.autograd.backward(ts, gs))
        for _, leaf in bounds[k]:
            leaf.grad = None
        after_stage(k)


class BucketReducer:
    """Async all-reduce(SUM) of contiguous gradient-arena buckets over a process group. `launch(k)` enqueues
    bucket k behind the work already on the current stream (ProcessGroupNCCL waits on it; gloo copies through
    the host); `wait()` makes the current stream wait for every launched bucket."""

    def __init__(self, arena, ranges, world_size, group=None, active=None):
        self.arena = arena
        self.ranges = list(ranges)
        self.world_size = world_size
        self.active = world_size > 1 if active is None else bool(active)  # True at world 1: a one-rank group
        self.group = group
        self.works = []
        self.launched = []

    def launch(self, k):
        lo, hi = self.ranges[k]
        self.launched.append(k)
        if not self.active or hi <= lo:
            return
        import torch.distributed as dist
        self.works.append(dist.all_reduce(self.arena[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                          async_op=True))

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
        done, self.launched = self.launched, []
        return done


# ---- process launch and group setup (one process per GPU) -------------------------------------------------------

def find_free_network_port() -> int:
    """A free TCP port on 127.0.0.1 for the rendezvous (utils/dist.py:13-22)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def generate_ddp_command(world_size, script, argv, port=None):
    """The command that re-runs `script argv` as `world_size` ranks on this node (utils/dist.py:56-66: the reference
    writes a temp trainer file and runs `python -m torch.distributed.run --nproc_per_node N --master_port P file`;
    here the script itself is re-run with its own arguments, so no temp file). Rendezvous on 127.0.0.1."""
    port = find_free_network_port() if port is None else int(port)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(world_size)}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(script), *[str(a) for a in argv]]


class LaunchError(RuntimeError):
    """A multi-GPU request this node or environment cannot satisfy (wrong GPU count / WORLD_SIZE mismatch)."""


def check_world(gpus, env=None, visible=None, share_gpu=False):
    """Validate a `--gpus N` request against the environment BEFORE any GPU call. Returns "launch" when N > 1 and
    this process is not a rank yet (the caller re-launches itself via generate_ddp_command), "rank" when it runs as
    one of N ranks (WORLD_SIZE == N), "single" for N == 1 outside a launcher. Raises LaunchError when WORLD_SIZE is
    set and differs from N, or when fewer than N GPUs are visible (`visible`: device count, default
    torch.cuda.device_count(), which does not initialise the GPU). share_gpu (tests only: gloo ranks placed on
    GPU rank % visible) needs one visible GPU."""
    env = os.environ if env is None else env
    gpus = int(gpus)
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise LaunchError(f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}: they must agree "
                              f"(run torch.distributed.run --nproc-per-node {gpus} ... --gpus {gpus}, or drop the "
                              f"launcher and let --gpus {gpus} start the ranks)")
        return "rank" if gpus > 1 else "single"
    if gpus == 1:
        return "single"
    n = torch.cuda.device_count() if visible is None else int(visible)
    if share_gpu and n >= 1:
        return "launch"
    if n < gpus:
        raise LaunchError(f"--gpus {gpus} asks for {gpus} ranks (one per GPU) but {n} GPU(s) are visible")
    return "launch"


def launch_ranks(world_size, script, argv):
    """Run `script argv` as world_size ranks in a CHILD process (never exec: trainer.py:184-204 runs the DDP command
    with subprocess.run as well) and return its exit code."""
    cmd = generate_ddp_command(world_size, script, argv)
    print(f"DDP: launching {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    env["ADR_SELF_LAUNCHED"] = "1"
    return subprocess.run(cmd, env=env).returncode


def setup_ddp(backend=None, timeout_s=10800, share_gpu=False):
    """Per-rank process-group setup (trainer.py:217-228): device = LOCAL_RANK, backend nccl (= RCCL on ROCm) when a
    GPU is there else gloo, with the reference's 3 h timeout. Returns (rank, local_rank, world_size, device).
    The reference also exports TORCH_NCCL_BLOCKING_WAIT=1; that makes every `work.wait()` block the host until the
    all-reduce finishes, which would stop the host from enqueueing the next stage-graph replay behind the bucket
    collectives (engine/ddp.py BucketReducer), so the timeout is left to the process group's watchdog instead.
    share_gpu (gloo only; tests on a one-GPU box): rank r uses GPU LOCAL_RANK % device_count."""
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() and dist.is_nccl_available() else "gloo"
    if share_gpu and backend == "nccl":
        raise LaunchError("share_gpu needs the gloo backend (RCCL refuses two ranks on one GPU)")
    if torch.cuda.is_available():
        gi = local % torch.cuda.device_count() if share_gpu else local
        torch.cuda.set_device(gi)
        dev = torch.device("cuda", gi)
    elif backend == "nccl":
        raise LaunchError("backend nccl (RCCL) needs a GPU")
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, timeout=timedelta(seconds=timeout_s), rank=rank, world_size=world, **kw)
    return rank, local, world, dev
