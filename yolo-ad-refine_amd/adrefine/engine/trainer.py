"""Training step for the AD-Refine hot path — the reference trainer's step semantics
(engine/trainer.py:383-398, optimizer_step :580-588, build_optimizer :753-813, ModelEMA torch_utils.py:521-546,
DDP :217-273) on libadr_hip:

  zero the flat fp32 gradient arena (one hipMemsetAsync)
  forward + v8DetectionLoss + backward   (HIP kernels; every parameter gradient is accumulated by its
                                          kernel straight into the arena — no per-parameter grad tensors)
  [DDP] all-reduce SUM of the arena over RCCL (== the reference's loss*world_size followed by DDP's average)
  clip_grad_norm_(10) + SGD(momentum, nesterov=True, 3 param groups) + EMA   (one fused multi-tensor pair)

The step can be captured once into HIP graphs (`capture(batch)`, torch.cuda.CUDAGraph over hipGraph): one graph
for zero + forward + loss + backward, one for the optimizer tail, with the RCCL all-reduce between them. Replay
costs two launches per step instead of ~2000 kernel launches from Python. Per-step scalars (lr per group,
EMA decay, first-step flag) live in a device vector written by a stream-ordered kernel before each replay.

Parameters that never receive a gradient (e.g. AdaptiveDynamicTanh.scale_weights, unused by the reference's
forward) are skipped by SGD exactly like torch.optim.SGD skips p.grad is None.
Mixed precision: the reference runs fp16 autocast + GradScaler; this build computes in bf16 (fp32 exponent
range), so no loss scaling is needed and the GradScaler is the identity.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from .. import kernels as K
from ..native import lib

_NORM_TYPES = tuple(v for k, v in nn.__dict__.items() if "Norm" in k and isinstance(v, type))
_ENTRY = np.dtype([("p", "<u8"), ("g", "<u8"), ("b", "<u8"), ("e", "<u8"), ("n", "<i8"), ("grp", "<i4"),
                   ("pad", "<i4")])
_CHUNK = np.dtype([("e", "<i4"), ("p", "<i4"), ("s", "<i8"), ("l", "<i8")])


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


class FusedTrainer:
    """One process per GPU. `step(batch)` = zero grads + fwd + loss + bwd (+ all-reduce) + clip + SGD + EMA;
    returns the loss items (device tensor, no host sync)."""

    CHUNK = 1 << 12  # elements per optimizer block: ~1.6k blocks for the n model (16 per thread, 4 in flight)

    def __init__(self, model, lr0=0.01, momentum=0.937, weight_decay=5e-4, nbs=64, batch_size=64, world_size=1,
                 process_group=None, ema=True, ema_decay=0.9999, ema_tau=2000, max_norm=10.0):
        self.model = model
        self.world_size = world_size
        self.pg = process_group
        self.momentum = momentum
        self.max_norm = max_norm
        accumulate = max(round(nbs / batch_size), 1)
        self.wd = weight_decay * batch_size * accumulate / nbs  # trainer.py:305-306
        self.lr = [lr0, lr0, lr0]
        self.dev = dev = next(model.parameters()).device
        groups = param_groups(model)
        self.entries = [(name, p, gi, True) for gi, lst in enumerate(groups) for name, p in lst]
        self.nparam = sum(p.numel() for _, p, _, _ in self.entries)
        self.grad = torch.zeros(self.nparam, dtype=torch.float32, device=dev)
        self.mom = torch.zeros(self.nparam, dtype=torch.float32, device=dev)
        off = 0
        self._goff = []
        for _, p, _, _ in self.entries:
            p._adr_grad = self.grad[off:off + p.numel()]
            p._adr_used = False
            self._goff.append(off)
            off += p.numel()
        # EMA over every floating state entry (params + BN running stats), buffers as group 3
        self.use_ema = ema
        pset = {id(p) for _, p, _, _ in self.entries}
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

    def forward_backward(self, batch):
        K.zero_(self.grad)
        self.model.train()
        with K.pack_scope(self.packs):
            self.packs.pack_all()  # every conv weight's bf16 operand copies, one launch (no-op on the first step)
            loss, items = self.model(batch)
            with K.defer_wgrad():  # conv weight-gradient split reductions: a few batched launches at the end
                loss.backward()
        return items

    def _set_hyper(self):
        d = self.ema_decay * (1 - math.exp(-(self.updates + 1) / self.ema_tau))
        vals = [self.lr[0], self.lr[1], self.lr[2], self.wd, 0.0, 0.0, self.momentum, 1.0,
                1.0 if self.updates == 0 else 0.0, d]
        arr = (ctypes.c_float * len(vals))(*vals)
        lib.adr_set_f32(K.fptr(self.hyper), ctypes.cast(arr, ctypes.c_void_p), len(vals), K.stream())

    def _allreduce(self):
        if self.world_size > 1:
            import torch.distributed as dist
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.pg)

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

    def step(self, batch):
        """zero grads + fwd + loss + bwd (+ all-reduce) + clip + SGD + EMA; returns the loss items (device)."""
        self._set_hyper()
        if self.graphs is not None:
            g_fb, g_opt, items = self.graphs
            if batch is not self.static_batch:
                b = self._prepare(batch)
                self.static_batch["img"].copy_(b["img"], non_blocking=True)
                gt, sgt = b["gt"], self.static_batch["gt"]
                if gt.shape[1] > sgt.shape[1]:
                    raise RuntimeError(f"captured step holds {sgt.shape[1]} targets per image, batch has {gt.shape[1]}")
                sgt.zero_()  # padded rows are masked out by the assigner (mask_gt), as the reference's own padding
                sgt[:, :gt.shape[1]].copy_(gt, non_blocking=True)
            g_fb.replay()
            self._allreduce()
            g_opt.replay()
        else:
            items = self.forward_backward(batch)
            self._allreduce()
            if self.tab_dev is None:  # the set of parameters that receive gradients is static: build once
                self._build_table()
            self._opt()
        self.packs.valid = False  # weights changed: the next forward repacks
        self.updates += 1
        return items.detach()

    def capture(self, batch, max_targets=None):
        """Capture the step into HIP graphs. Call after at least one eager step (lazy caches, the parameter
        table). The batch becomes the graph's static input (targets padded to max_targets per image); later
        `step(b)` copies b into it."""
        assert self.tab_dev is not None, "run one eager step before capture()"
        b = self._prepare(batch)
        gt = b["gt"]
        cap = max(max_targets or gt.shape[1], gt.shape[1])
        sgt = torch.zeros(gt.shape[0], cap, 5, dtype=torch.float32, device=self.dev)
        sgt[:, :gt.shape[1]].copy_(gt)
        self.static_batch = {"img": b["img"].clone(), "gt": sgt}
        # warm-up on the capture side stream mutates BN running stats: snapshot and restore them
        bufs = list(self.model.buffers())
        saved = [t.clone() for t in bufs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.forward_backward(self.static_batch)
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip(bufs, saved):
            t.copy_(v)
        g_fb, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            items = self.forward_backward(self.static_batch)
        with torch.cuda.graph(g_opt):
            self._opt()
        self.graphs = (g_fb, g_opt, items)
        torch.cuda.synchronize()
        return self.static_batch

    def param_grad(self, name):
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
