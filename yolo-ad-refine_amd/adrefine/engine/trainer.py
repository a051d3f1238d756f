"""Training step for the AD-Refine hot path — the reference trainer's step semantics
(engine/trainer.py:305-306 accumulate / weight-decay scaling, :330 + :369-381 warm-up, :383-398 step loop,
optimizer_step :580-588, build_optimizer :753-813, LambdaLR :209-215, ModelEMA torch_utils.py:521-546,
DDP :217-273) on libadr_hip:

  forward + v8DetectionLoss + backward   (HIP kernels; every parameter gradient is accumulated by its kernel
                                          straight into one flat fp32 arena — no per-parameter grad tensors)
  [DDP] bucketed all-reduce SUM of the arena over RCCL, overlapped with the backward (engine/ddp.py)
  every `accumulate` batches (ni - last_opt_step >= accumulate, trainer.py:396):
      clip_grad_norm_(10) + SGD(momentum, nesterov=True, 3 param groups) + EMA + zero_grad   (one fused pair)

`batch_size` is the reference's `self.batch_size` = args.batch, the GLOBAL batch over all ranks
(trainer.py:290 divides it per rank); accumulate = max(round(nbs / batch_size), 1) and
weight_decay *= batch_size * accumulate / nbs exactly as trainer.py:305-306.

Warm-up / schedule (`nb` = batches per epoch given): for ni <= nw = max(round(warmup_epochs * nb), 100) the
accumulate count, the per-group lr (bias group from warmup_bias_lr, others from 0, towards lr0 * lf(epoch)) and
the momentum (from warmup_momentum) are interpolated per batch as trainer.py:369-381; afterwards lr follows the
LambdaLR factor lf(epoch) (linear, or one_cycle with cos_lr). Without `nb` the schedule is constant
(lr0, momentum, the setup accumulate) — the benchmark's steady state.

The step can be captured once into HIP graphs (`capture(batch)`, torch.cuda.CUDAGraph over hipGraph): the
forward + loss + backward (one graph per backward stage when the step is staged for DDP) and the optimizer tail,
with the collectives launched between replays. Per-step scalars (lr per group, momentum, EMA decay, first-step
flag) live in a device vector written by a stream-ordered kernel before each replay.

Parameters that never receive a gradient (e.g. AdaptiveDynamicTanh.scale_weights, unused by the reference's
forward) are skipped by SGD exactly like torch.optim.SGD skips p.grad is None.
Mixed precision: the reference runs fp16 autocast + GradScaler; this build computes in bf16 (fp32 exponent
range), so no loss scaling is needed and the GradScaler is the identity.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch
import torch.nn as nn

from .. import kernels as K
from ..native import lib
from .ddp import BucketReducer, cuts_for_bucket, layer_of, stage_of, staged_backward

# Graph capture in thread-local mode: with a process group up (DDP, or bench.py's one-GPU RCCL leg), the RCCL
# watchdog thread polls its work events while this thread captures; in torch's default global mode that query
# fails the capture ("operation not permitted when stream is capturing") and takes the process down
_CAPTURE_MODE = "thread_local"
_NORM_TYPES = tuple(v for k, v in nn.__dict__.items() if "Norm" in k and isinstance(v, type))
_ENTRY = np.dtype([("p", "<u8"), ("g", "<u8"), ("b", "<u8"), ("e", "<u8"), ("n", "<i8"), ("grp", "<i4"),
                   ("pad", "<i4")])
_CHUNK = np.dtype([("e", "<i4"), ("p", "<i4"), ("s", "<i8"), ("l", "<i8")])
# stage ends for the bucketed all-reduce: buckets of ~ADR_DDP_BUCKET_MB MB of gradients, filled from the last layer
# down (ddp.cuts_for_bucket); DDP_CUTS overrides with fixed layer cuts (e.g. "6,10"). 8 MB: one cut after L10, two
# stages — the first bucket (L11-L33, 8.5 MiB of 15.6) all-reduces under the backbone's backward. Measured on one GPU with
# the one-rank RCCL group (scripts/_r06l.sh, same box): 4 MB buckets (cuts 7, 10, 20) cost 2.0 % over the unstaged
# step, 8 MB 0.9 %, 16 MB (no cut, no overlap) 0.3 %; SURVEY §8e puts the 16.4 MB all-reduce at 30-60 us over xGMI,
# so the exposed second bucket costs about what the extra cuts would
DDP_BUCKET_MB = float(os.environ.get("ADR_DDP_BUCKET_MB", "8"))
DDP_CUTS = tuple(int(v) for v in os.environ["ADR_DDP_CUTS"].split(",")) if os.environ.get("ADR_DDP_CUTS") else None


def param_groups(model):
    """build_optimizer grouping (trainer.py:781-789): 'bias' in name -> g2; norm-layer weights -> g1; else g0."""
    g = [], [], []
    for mname, module in model.named_modules():
        for pname, p in module.named_parameters(recurse=False):
            if not p.requires_grad:
                continue
            full = f"{mname}.{pname}" if mname else pname
            if "bias" in full:
                g[2].append((full, p))
            elif isinstance(module, _NORM_TYPES):
                g[1].append((full, p))
            else:
                g[0].append((full, p))
    return g


class Schedule:
    """lr / momentum / accumulate per batch index ni (trainer.py:209-215, 305, 330, 369-381). Trainer group
    order is (g0 decayed weights, g1 norm weights, g2 biases); the reference's optimizer param_groups are
    (g2, g0, g1), so its `j == 0` warm-up bias rule applies to g2 here."""

    def __init__(self, lr0=0.01, lrf=0.01, momentum=0.937, nbs=64, batch_size=64, epochs=100, nb=None,
                 warmup_epochs=3.0, warmup_bias_lr=0.1, warmup_momentum=0.8, cos_lr=False):
        self.lr0, self.lrf, self.momentum, self.epochs, self.nb = lr0, lrf, momentum, epochs, nb
        self.cos_lr = cos_lr
        self.warmup_bias_lr, self.warmup_momentum = warmup_bias_lr, warmup_momentum
        self.acc_target = nbs / batch_size
        self.accumulate0 = max(round(nbs / batch_size), 1)  # trainer.py:305
        self.nw = (max(round(warmup_epochs * nb), 100) if warmup_epochs > 0 else -1) if nb else -1  # :330

    def lf(self, epoch):
        if self.cos_lr:  # utils/__init__.py one_cycle(1, lrf, epochs)
            return ((1 - math.cos(epoch * math.pi / self.epochs)) / 2) * (self.lrf - 1) + 1
        return max(1 - epoch / self.epochs, 0) * (1.0 - self.lrf) + self.lrf  # trainer.py:214

    def at(self, ni):
        """(lrs (g0, g1, g2), momentum, accumulate) in effect for batch ni."""
        if self.nb is None:
            return [self.lr0] * 3, self.momentum, self.accumulate0
        epoch = ni // self.nb
        target = self.lr0 * self.lf(epoch)
        if ni <= self.nw:
            xi = [0, self.nw]
            acc = max(1, int(np.interp(ni, xi, [1, self.acc_target]).round()))
            lr_bias = float(np.interp(ni, xi, [self.warmup_bias_lr, target]))
            lr_w = float(np.interp(ni, xi, [0.0, target]))
            mom = float(np.interp(ni, xi, [self.warmup_momentum, self.momentum]))
            return [lr_w, lr_w, lr_bias], mom, acc
        if self.nw >= 0:  # after warm-up accumulate keeps its last interpolated value
            acc = max(1, int(np.interp(self.nw, [0, self.nw], [1, self.acc_target]).round()))
        else:
            acc = self.accumulate0
        return [target] * 3, self.momentum, acc


class FusedTrainer:
    """One process per GPU. `step(batch)` = fwd + loss + bwd (+ bucketed all-reduce) and, every `accumulate`
    batches, clip + SGD + EMA + zero_grad; returns the loss items (device tensor, no host sync)."""

    CHUNK = 1 << 12  # elements per optimizer block: ~1.6k blocks for the n model (16 per thread, 4 in flight)

    def __init__(self, model, lr0=0.01, momentum=0.937, weight_decay=5e-4, nbs=64, batch_size=64, world_size=1,
                 process_group=None, ema=True, ema_decay=0.9999, ema_tau=2000, max_norm=10.0, epochs=100, nb=None,
                 lrf=0.01, warmup_epochs=3.0, warmup_bias_lr=0.1, warmup_momentum=0.8, cos_lr=False, stages=None,
                 collectives=None):
        self.model = model
        self.world_size = world_size
        # collectives=True issues the bucket all-reduces even at world_size 1 (a one-rank RCCL group exercises the
        # same interleaving of stage-graph replays and eager collectives as the multi-GPU step)
        self.collectives = world_size > 1 if collectives is None else bool(collectives)
        self.pg = process_group
        self.max_norm = max_norm
        self.batch_size = batch_size
        self.sched = Schedule(lr0, lrf, momentum, nbs, batch_size, epochs, nb, warmup_epochs, warmup_bias_lr,
                              warmup_momentum, cos_lr)
        self.accumulate = self.sched.accumulate0
        self.wd = weight_decay * batch_size * self.accumulate / nbs  # trainer.py:305-306
        self.lr, self.momentum, _ = self.sched.at(0)
        self.ni, self.last_opt_step = 0, -1
        # backward stages: DDP overlaps bucket all-reduces with the remaining stages (engine/ddp.py)
        if stages is None:
            stages = (DDP_CUTS if DDP_CUTS is not None else cuts_for_bucket(model, DDP_BUCKET_MB)) \
                if self.collectives else ()
        self.cuts = tuple(stages)
        self.dev = dev = next(model.parameters()).device
        groups = param_groups(model)
        plist = [(name, p, gi) for gi, lst in enumerate(groups) for name, p in lst]
        # arena order: stage-major, LAST stage first (its gradients are final first), group order within a stage
        nst = len(self.cuts) + 1
        plist.sort(key=lambda e: nst - 1 - stage_of(layer_of(e[0]), self.cuts))
        self.entries = [(name, p, gi, True) for name, p, gi in plist]
        self.nparam = sum(p.numel() for _, p, _, _ in self.entries)
        self.grad = torch.zeros(self.nparam, dtype=torch.float32, device=dev)
        self.mom = torch.zeros(self.nparam, dtype=torch.float32, device=dev)
        off = 0
        self._goff = []
        bounds = [[None, None] for _ in range(nst)]
        for name, p, _, _ in self.entries:
            p._adr_grad = self.grad[off:off + p.numel()]
            p._adr_used = False
            self._goff.append(off)
            s = stage_of(layer_of(name), self.cuts)
            if bounds[s][0] is None:
                bounds[s][0] = off
            off += p.numel()
            bounds[s][1] = off
        self.buckets = [(b[0] or 0, b[1] or 0) for b in bounds]  # arena range of each stage's gradients
        self.reducer = BucketReducer(self.grad, self.buckets, world_size, process_group, active=self.collectives)
        # EMA over every floating state entry (params + BN running stats), buffers as group 3
        self.use_ema = ema
        pset = {id(p) for _, p, _, _ in self.entries}
        # integer buffers (BN num_batches_tracked) as the reference's EMA copy holds them: never updated
        self.ema_int = {k: v.detach().clone() for k, v in model.state_dict().items() if not v.dtype.is_floating_point}
        for k, v in model.state_dict(keep_vars=True).items():
            if v.dtype.is_floating_point and id(v) not in pset:
                self.entries.append((k, v, 3, False))
                self._goff.append(-1)
        ntot = sum(t.numel() for _, t, _, _ in self.entries)
        self.ema_flat = torch.empty(ntot, dtype=torch.float32, device=dev) if ema else None
        self._eoff, chunks, off = [], [], 0
        for ei, (_, t, _, _) in enumerate(self.entries):
            self._eoff.append(off)
            n = t.numel()
            for s in range(0, n, self.CHUNK):
                chunks.append((ei, 0, s, min(self.CHUNK, n - s)))
            if ema:
                self.ema_flat[off:off + n].copy_(t.detach().reshape(-1))
            off += n
        self.nchunks = len(chunks)
        assert lib.adr_opt_entry_size() == _ENTRY.itemsize and lib.adr_opt_chunk_size() == _CHUNK.itemsize
        self.chunks_dev = torch.from_numpy(np.array(chunks, dtype=_CHUNK).view(np.uint8).copy()).to(dev)
        self.partial = torch.empty(self.nchunks, dtype=torch.float32, device=dev)
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.tab_dev = None
        self.updates = 0
        self.ema_decay = ema_decay
        self.ema_tau = ema_tau
        self.hyper = torch.zeros(16, dtype=torch.float32, device=dev)
        self.graphs = None
        self._sets = {}  # target capacity -> (graphs, static batch): one captured step per capacity bucket
        self.packs = K.PackCache()

    def _build_table(self):
        tab = np.zeros(len(self.entries), dtype=_ENTRY)
        for ei, (_, t, g, isp) in enumerate(self.entries):
            used = isp and getattr(t, "_adr_used", False)
            tab["p"][ei] = t.data_ptr()
            tab["g"][ei] = self.grad.data_ptr() + 4 * self._goff[ei] if used else 0
            tab["b"][ei] = self.mom.data_ptr() + 4 * self._goff[ei] if isp else 0
            tab["e"][ei] = self.ema_flat.data_ptr() + 4 * self._eoff[ei] if self.use_ema else 0
            tab["n"][ei] = t.numel()
            tab["grp"][ei] = g if used else 3
        self.tab_dev = torch.from_numpy(tab.view(np.uint8).copy()).to(self.dev)

    def forward_backward(self, batch, after_stage=None):
        """fwd + loss + bwd, accumulating into the arena (zeroed by the optimizer step, as zero_grad at
        trainer.py:586). With stages, `after_stage(s)` runs as soon as stage s's gradients are final."""
        self.model.train()
        with K.pack_scope(self.packs):
            self.packs.pack_all()  # every conv weight's bf16 operand copies, one launch (no-op on the first step)
            if not self.cuts:
                loss, items = self.model(batch)
                with K.defer_wgrad():  # conv weight-gradient split reductions: a few batched launches at the end
                    loss.backward()
                if after_stage is not None:
                    after_stage(0)
                return items
            loss, items = self.model.loss(batch, cuts=self.cuts)
            bounds = self.model.stage_bounds
            self.model.stage_bounds = None

            def run(fn):
                with K.defer_wgrad():
                    fn()
            staged_backward(loss, bounds, run, after_stage or (lambda s: None))
        return items

    def _set_hyper(self):
        d = self.ema_decay * (1 - math.exp(-(self.updates + 1) / self.ema_tau))
        vals = [self.lr[0], self.lr[1], self.lr[2], self.wd, 0.0, 0.0, self.momentum, 1.0,
                1.0 if self.updates == 0 else 0.0, d]
        arr = (ctypes.c_float * len(vals))(*vals)
        lib.adr_set_f32(K.fptr(self.hyper), ctypes.cast(arr, ctypes.c_void_p), len(vals), K.stream())

    def _opt(self):
        lib.adr_opt_step(K.fptr(self.tab_dev), K.fptr(self.chunks_dev), self.nchunks, K.fptr(self.partial),
                         float(self.max_norm), K.fptr(self.hyper), K.fptr(self.norm), K.stream())

    def _prepare(self, batch):
        """{'img', 'gt'} on the device; 'gt' (B, nmax, 5) built from the collate_fn keys when absent."""
        img = batch["img"]
        gt = batch.get("gt")
        if gt is None:
            from ..utils.loss import preprocess_targets
            gt = preprocess_targets(batch["batch_idx"], batch["cls"], batch["bboxes"], img.shape[0],
                                    (img.shape[2], img.shape[3]))
        return {"img": img.to(self.dev, non_blocking=True), "gt": gt.to(self.dev, non_blocking=True).float()}

    def will_step(self):
        """Whether the next step() runs the optimizer (ni - last_opt_step >= accumulate, trainer.py:396)."""
        _, _, acc = self.sched.at(self.ni)
        return self.ni - self.last_opt_step >= acc

    def step(self, batch):
        """fwd + loss + bwd (+ all-reduce) and, when due, clip + SGD + EMA + zero_grad; returns the loss items
        (device). The all-reduce runs only on batches that end in an optimizer step: the gradient sum is linear,
        so reducing the accumulated arena once equals DDP's reduction on every backward."""
        self.lr, self.momentum, self.accumulate = self.sched.at(self.ni)
        opt_now = self.ni - self.last_opt_step >= self.accumulate
        reduce_now = opt_now and self.collectives
        if opt_now:
            self._set_hyper()
        if self.graphs is not None:
            if batch is not self.static_batch:
                b = self._prepare(batch)
                gt = b["gt"]
                self._select_capacity(gt.shape[1], b)  # the smallest captured target capacity that holds the batch
                self.static_batch["img"].copy_(b["img"], non_blocking=True)
                sgt = self.static_batch["gt"]
                sgt.zero_()  # padded rows are masked out by the assigner (mask_gt), as the reference's own padding
                sgt[:, :gt.shape[1]].copy_(gt, non_blocking=True)
            g_stages, g_opt, items = self.graphs
            for i, g in enumerate(g_stages):  # stage S-1 (with the forward) first, stage 0 last
                g.replay()
                if reduce_now:
                    self.reducer.launch(len(g_stages) - 1 - i)
            if reduce_now:
                self.reducer.wait()
            if opt_now:
                g_opt.replay()
        else:
            items = self.forward_backward(batch, self.reducer.launch if reduce_now else None)
            if reduce_now:
                self.reducer.wait()
            if self.tab_dev is None:  # the set of parameters that receive gradients is static: build once
                self._build_table()
            if opt_now:
                self._opt()
        if opt_now:
            self.packs.valid = False  # weights changed: the next forward repacks
            self.updates += 1
            self.last_opt_step = self.ni
        self.ni += 1
        return items.detach()

    @staticmethod
    def capacity_bucket(n):
        """Target capacity captured for a batch with n targets per image: the next power of two (at least 8), so a
        real dataloader (Poisson-like label counts, up to ~100 per image on COCO) needs a handful of captures."""
        return max(8, 1 << max(0, int(n) - 1).bit_length())

    def _select_capacity(self, need, b):
        """Activate the captured step with the smallest per-image target capacity >= need; capture one for
        capacity_bucket(need) (from this batch) when none holds it (capture() then drops the smaller sets). The
        reference pads targets per batch (utils/loss.py:392-408); the padded rows are masked by the assigner, so
        the capacity does not change the step's result — a larger batch never fails mid-training."""
        if need <= self.static_batch["gt"].shape[1] and need > self._cap_floor():
            return
        fits = [c for c in self._sets if c >= need]
        if fits:
            self.graphs, self.static_batch = self._sets[min(fits)]
            return
        self.capture(b, max_targets=self.capacity_bucket(need))

    def _cap_floor(self):
        """Largest captured capacity below the active one (a batch above it keeps the active set)."""
        cur = self.static_batch["gt"].shape[1]
        lower = [c for c in self._sets if c < cur]
        return max(lower) if lower else -1

    def capture(self, batch, max_targets=None):
        """Capture the step into HIP graphs. Call after at least one eager step (lazy caches, the parameter
        table). The batch becomes the graph's static input (targets padded to max_targets per image); later
        `step(b)` copies b into it. The capture is kept keyed by its target capacity; the first batch that exceeds
        it captures a larger bucket (capacity_bucket), which replaces every smaller one."""
        assert self.tab_dev is not None, "run one eager step before capture()"
        b = self._prepare(batch)
        gt = b["gt"]
        cap = max(max_targets or gt.shape[1], gt.shape[1])
        sgt = torch.zeros(gt.shape[0], cap, 5, dtype=torch.float32, device=self.dev)
        sgt[:, :gt.shape[1]].copy_(gt)
        self.static_batch = {"img": b["img"].clone(), "gt": sgt}
        # warm-up on the capture side stream mutates BN running stats and the arena: snapshot / restore them
        bufs = list(self.model.buffers())
        saved = [t.clone() for t in bufs]
        gsaved = self.grad.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.forward_backward(self.static_batch)
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip(bufs, saved):
            t.copy_(v)
        nst = len(self.cuts) + 1
        g_stages = [torch.cuda.CUDAGraph() for _ in range(nst)]
        cm = [torch.cuda.graph(g_stages[0], capture_error_mode=_CAPTURE_MODE)]
        cm[0].__enter__()
        nxt = [1]

        def after_stage(s):  # close this stage's graph, open the next one on the same memory pool
            cm[0].__exit__(None, None, None)
            if nxt[0] < nst:
                cm[0] = torch.cuda.graph(g_stages[nxt[0]], pool=g_stages[0].pool(), capture_error_mode=_CAPTURE_MODE)
                nxt[0] += 1
                cm[0].__enter__()

        try:
            items = self.forward_backward(self.static_batch, after_stage)
        except BaseException:
            if nxt[0] <= nst:
                try:
                    cm[0].__exit__(None, None, None)
                except Exception:  # noqa: BLE001 - capture already broken; surface the original error
                    pass
            raise
        g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_opt, pool=g_stages[0].pool(), capture_error_mode=_CAPTURE_MODE):
            self._opt()
        self.graphs = (g_stages, g_opt, items)
        # a larger capacity holds every batch a smaller one held: drop the smaller sets, so graph memory stays at
        # ONE captured step (each set owns a private pool with a whole step's activations) however many buckets a
        # real dataloader walks through
        dropped = [c for c in self._sets if c < cap]
        for c in dropped:
            del self._sets[c]
        self._sets[cap] = (self.graphs, self.static_batch)
        self.grad.copy_(gsaved)
        torch.cuda.synchronize()
        if dropped:
            torch.cuda.empty_cache()  # return the dropped sets' private pools
        return self.static_batch

    def param_grad(self, name):
        """View of a parameter's slice of the gradient arena (valid between backward and the optimizer step)."""
        for ei, (n, t, _, isp) in enumerate(self.entries):
            if n == name and isp:
                return self.grad[self._goff[ei]:self._goff[ei] + t.numel()].view(t.shape)
        raise KeyError(name)

    def ema_state_dict(self):
        out = {}
        for ei, (name, t, _, _) in enumerate(self.entries):
            off = self._eoff[ei]
            out[name] = self.ema_flat[off:off + t.numel()].view(t.shape)
        return out
