"""Model graph: yaml -> module list, and the forward driver — drop-in for the reference's
ultralytics/nn/tasks.py (parse_model :943-1108, DetectionModel :309-398, BaseModel._predict_once :141-168).

The channel arithmetic, repeat handling, `head_channel` / `fusion_mode` string resolution and the
per-module argument rules are restated from parse_model, so the reference's z-yaml configs build the same
layers with the same state_dict keys (541 for the 701 yaml). Layer classes resolve to the HIP-backed modules
of adrefine.nn.modules; `nn.X` rows resolve to the HIP drop-ins for nn.Conv2d / nn.ConvTranspose2d.
"""
from __future__ import annotations

import ast
import contextlib
import math
import re
from copy import deepcopy
from pathlib import Path

import torch
import torch.nn as nn
import yaml

from .. import kernels as K
from .modules import block, conv, head

# name -> class, mirroring the reference's tasks.py import list for the modules on this path
_REGISTRY = {
    "Conv": conv.Conv, "Bottleneck": block.Bottleneck, "C2f": block.C2f, "C3": block.C3, "C3k2": block.C3k2,
    "SPPF": block.SPPF, "C3k2_MLCA": block.C3k2_MLCA, "C2PTSSA": block.C2PTSSA, "C2PSA": block.C2PSA,
    "ELA_HSFPN": block.ELA_HSFPN, "Multiply": block.Multiply, "Add": block.Add, "Fusion": block.Fusion,
    "AYHead": head.AYHead, "AYHead1": head.AYHead1, "C2TSSA_DYT_Mona_EDFFN": block.C2TSSA_DYT_Mona_EDFFN,
    "Detect": head.Detect, "DWConv": conv.DWConv, "Concat": conv.Concat,
}
_NN = {"Conv2d": conv.Conv2d, "ConvTranspose2d": conv.ConvTranspose2d, "Upsample": conv.Upsample}

_CH_MODULES = {"Conv", "DWConv", "Bottleneck", "SPPF", "C2f", "C3", "C3k2", "C3k2_MLCA", "C2PTSSA", "C2PSA",
               "C2TSSA_DYT_Mona_EDFFN", "nn.Conv2d", "nn.ConvTranspose2d"}
_REPEAT_MODULES = {"C2f", "C3", "C3k2", "C3k2_MLCA", "C2PTSSA", "C2PSA", "C2TSSA_DYT_Mona_EDFFN"}


def register(name, cls):
    """Register an extra module class for yaml lookup (e.g. the 697 Mona variant)."""
    _REGISTRY[name] = cls


def make_divisible(x, divisor):
    if isinstance(divisor, torch.Tensor):
        divisor = int(divisor.max())
    return math.ceil(x / divisor) * divisor


def guess_model_scale(model_path):
    """tasks.py:1140-1155."""
    with contextlib.suppress(AttributeError):
        return re.search(r"yolo[v]?\d+([nslmx])", Path(model_path).stem).group(1)
    return ""


def yaml_model_load(path):
    """tasks.py:1110-1124 (without the hub download / -p6 renames): dict + scale guessed from the file name;
    a scaled name resolves to its unified file (yolo11n.yaml -> yolo11.yaml, scale 'n')."""
    path = Path(path)
    unified = Path(re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", str(path)))
    d = yaml.safe_load((unified if unified.is_file() else path).read_text())
    d["scale"] = guess_model_scale(path)
    d["yaml_file"] = str(path)
    return d


def _resolve(m):
    if m.startswith("nn."):
        name = m[3:]
        if name in _NN:
            return _NN[name]
        raise NotImplementedError(f"{m}: no HIP drop-in on the AD-Refine hot path")
    if m not in _REGISTRY:
        raise NotImplementedError(f"module '{m}' is not on the AD-Refine hot path (registered: {sorted(_REGISTRY)})")
    return _REGISTRY[m]


def parse_model(d, ch, verbose=False):
    """Restatement of the reference parse_model (tasks.py:943-1108) for the modules this build provides."""
    nc, scales = d.get("nc"), d.get("scales")
    head_channel, fusion_mode = d.get("head_channel"), d.get("fusion_mode")
    depth, width = d.get("depth_multiple", 1.0), d.get("width_multiple", 1.0)
    max_channels = float("inf")
    scale = d.get("scale")
    if scales:
        if not scale:
            scale = tuple(scales.keys())[0]  # tasks.py:952-957 (the reference warns and assumes the first)
        depth, width, max_channels = scales[scale]
    local = {"nc": nc, "head_channel": head_channel, "fusion_mode": fusion_mode}
    ch = [ch]
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
        mod = _resolve(m)
        args = list(args)
        for j, a in enumerate(args):
            if isinstance(a, str):
                with contextlib.suppress(ValueError):
                    args[j] = local[a] if a in local else ast.literal_eval(a)
        n = n_ = max(round(n * depth), 1) if n > 1 else n
        if m in _CH_MODULES:
            c1, c2 = ch[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2, *args[1:]]
            if m in _REPEAT_MODULES:
                args.insert(2, n)
                n = 1
            if m == "C3k2" and scale in "mlx":
                args[3] = True
        elif m == "ELA_HSFPN":
            args = [ch[f], *args]
            c2 = ch[f]
        elif m in ("Multiply", "Add"):
            c2 = ch[f[0]]
        elif m == "Fusion":
            inc = [ch[x] for x in f]
            args.insert(0, inc)
            mode = args[1] if len(args) > 1 else "bifpn"
            c2 = sum(inc) if mode == "concat" else inc[0]
        elif m == "Concat":
            c2 = sum(ch[x] for x in f)
        elif m in ("AYHead", "AYHead1", "Detect"):
            args.append([ch[x] for x in f])
        else:
            c2 = ch[f]
        m_ = nn.Sequential(*(mod(*args) for _ in range(n))) if n > 1 else mod(*args)
        t = m
        m_.np = sum(x.numel() for x in m_.parameters())
        m_.i, m_.f, m_.type = i, f, t
        if verbose:
            print(f"{i:>3}{str(f):>20}{n_:>3}{m_.np:10.0f}  {t:<45}{str(args):<30}")
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


def layer_strides(layers, ch_stride=1.0):
    """Output stride of every layer of a parsed model, from the convolution / upsample strides along its inputs —
    what the reference measures with a zero-image probe forward (tasks.py:333-346)."""
    out = []
    for m in layers:
        f = m.f
        s_in = (out[f] if f != -1 else (out[-1] if out else ch_stride)) if isinstance(f, int) else \
            (out[f[0]] if f[0] != -1 else out[-1])
        if isinstance(m, (conv.Conv, conv.Conv2d)):
            cv = m.conv if isinstance(m, conv.Conv) else m
            s_in = s_in * cv.stride[0]
        elif isinstance(m, conv.ConvTranspose2d):
            s_in = s_in / m.stride[0]
        elif isinstance(m, conv.Upsample):
            sf = m.scale_factor[0] if isinstance(m.scale_factor, tuple) else m.scale_factor
            s_in = s_in / float(sf)
        out.append(s_in)
    return out


def emulate_stride_probe(model):
    """The reference's stride probe (tasks.py:345) is a train-mode forward of a zero image BEFORE
    initialize_weights: every BatchNorm sees an all-zero batch (each conv has no bias and every block maps 0 to 0),
    so with torch's default momentum 0.1 it leaves running_mean 0, running_var 0.9 * running_var and
    num_batches_tracked 1. Reproduced here without running a forward."""
    for mm in model.modules():
        if isinstance(mm, nn.BatchNorm2d):
            mm.running_mean.mul_(0.9)
            mm.running_var.mul_(0.9)
            mm.num_batches_tracked += 1


def initialize_weights(model):
    """torch_utils.py:426-436: BatchNorm2d eps 1e-3 / momentum 0.03 (already the defaults of this build's BNs)."""
    for m in model.modules():
        if type(m) is nn.BatchNorm2d:
            m.eps, m.momentum = 1e-3, 0.03


def consumer_counts(layers):
    """How many later layers read each layer's output (its `f` references, -1 = the previous layer)."""
    uses = {}
    for m in layers:
        for j in ([m.f] if isinstance(m.f, int) else m.f):
            src = m.i - 1 if j == -1 else (j if j >= 0 else m.i + j)
            uses[src] = uses.get(src, 0) + 1
    return uses


def lazy_pair(m, n, save, cuts, uses):
    """Layer m ends in a Conv (a Conv row, or a C2f / C3k2 / SPPF / C2PSA block whose last op is its cv2) and only
    the next layer n reads its output, first through a Conv on the whole tensor (a Conv row, or the cv1 of C2f /
    SPPF / C2PSA): m's last BN-act is handed to that conv lazily — it applies the BN-act while staging
    (kernels.BnFwd) and, being the only reader, its data gradient is the BN's whole dz (kernels.BnStat)."""
    from .modules.block import C2f, C2PSA, SPPF
    from .modules.conv import Conv
    producer = type(m) is Conv or isinstance(m, (C2f, SPPF, C2PSA))
    return (producer and m.training and n is not None and n.f == -1 and m.i not in save and m.i not in cuts and
            (uses or {}).get(m.i, 1) == 1 and (type(n) is Conv or isinstance(n, (C2f, SPPF, C2PSA))))


def route_layers(layers, save, x, y, start=0, cuts=(), uses=None):
    """The layer loop of _predict_once (tasks.py:155-167): each layer reads x (f == -1) or saved outputs y[f],
    and its output is kept in y when a later layer reads it. An output read by several layers is handed to each
    reader as its own view (K.fanout), so its gradient is summed by one libadr launch instead of autograd adds.
    With `cuts`, the tensors crossing the end of each listed layer are replaced by detached leaves
    (engine/ddp.cut_live) and returned as per-cut (tensor, leaf) lists, so the backward can run stage by stage."""
    bounds = []
    views = {}
    if cuts:
        from ..engine.ddp import cut_live

    def fan(j, t):
        n = uses.get(j, 1) if uses else 1
        if n > 1 and torch.is_tensor(t) and t.dim() == 4 and t.requires_grad:
            views[j] = list(K.fanout(t, n))

    def take(j, t):
        v = views.get(j)
        return v.pop() if v else t

    if start > 0:
        fan(start - 1, x)
    from .modules.block import Add, Multiply
    nxt = {m.i: layers[k + 1] for k, m in enumerate(layers[:-1])}

    class _MulPend:  # a Multiply whose only reader is the next layer's two-input Add: computed there as one FMA
        __slots__ = ("a", "b")

        def __init__(self, a, b):
            self.a, self.b = a, b

    def mul_into_add(m):
        """Multiply (block.py:1442) feeding only the next layer's Add (block.py:1448) of two inputs — the HS-FPN
        gate-and-residual pair (yaml layers 17-18, 24-25): Add(Multiply(p, q), r) in one K.mul_add pass (bitwise the
        pair: the product rounded first)."""
        n = nxt.get(m.i)
        return (type(m) is Multiply and isinstance(m.f, list) and len(m.f) == 2 and n is not None and type(n) is Add
                and isinstance(n.f, list) and len(n.f) == 2 and (-1 in n.f or m.i in n.f) and m.i not in save
                and m.i not in cuts and (uses or {}).get(m.i, 1) == 1)

    def lazy_ok(m):
        return lazy_pair(m, nxt.get(m.i), save, cuts, uses)

    for m in layers[start:]:
        if m.f == -1:
            x = take(m.i - 1, x)
        elif isinstance(m.f, int):
            x = take(m.f, y[m.f])
        else:
            x = [take(m.i - 1, x) if j == -1 else take(j, y[j]) for j in m.f]
        if mul_into_add(m):
            x = _MulPend(x[0], x[1])
        elif isinstance(x, list) and any(isinstance(t, _MulPend) for t in x):
            pm = next(t for t in x if isinstance(t, _MulPend))
            x = K.mul_add(pm.a, pm.b, next(t for t in x if t is not pm))
        else:
            x = m(x, lazy=True) if lazy_ok(m) else m(x)
        y.append(x if m.i in save else None)
        if m.i in cuts:
            x = cut_live(x, y, layers, m.i, bounds)  # y[i] and x stay one leaf when they are one tensor
            if y[m.i] is not None:  # the next layer reads a saved index, not -1: x must still become the leaf,
                x = y[m.i]          # or the fan-out below would hand later stages views of the pre-cut tensor
            for j, vs in views.items():  # readers after the cut take views of the new leaves
                if vs:
                    views[j] = list(K.fanout(y[j], len(vs))) if len(vs) > 1 else [y[j]]
        fan(m.i, x)
    return x, bounds


class DetectionModel(nn.Module):
    """YOLO detection model (tasks.py:309-398). Compute dtype: float32 (parity) or bfloat16 (performance);
    parameters stay fp32. Input: float images (B, 3, H, W) in [0, 1] on a ROCm device."""

    def __init__(self, cfg="yolo11-701-YOLO-AD-Refine.yaml", ch=3, nc=None, verbose=False, compute_dtype=torch.float32):
        super().__init__()
        self.yaml = cfg if isinstance(cfg, dict) else yaml_model_load(cfg)
        ch = self.yaml["ch"] = self.yaml.get("ch", ch)
        if nc and nc != self.yaml["nc"]:
            self.yaml["nc"] = nc
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=ch, verbose=verbose)
        self.names = {i: f"{i}" for i in range(self.yaml["nc"])}
        self.inplace = self.yaml.get("inplace", True)
        m = self.model[-1]
        if isinstance(m, head.AYHead1):
            # AYHead is not a Detect subclass: the reference skips the stride probe (tasks.py:335) and the head
            # sets [8, 16, 32] itself (head.py:1209-1211)
            self.stride = m.stride
        elif isinstance(m, head.Detect):
            st = layer_strides(self.model)
            m.stride = torch.tensor([st[j] for j in m.f], dtype=torch.float32)
            self.stride = m.stride
            emulate_stride_probe(self)
            m.bias_init()
        else:
            self.stride = torch.Tensor([32])
        initialize_weights(self)
        self.compute_dtype = compute_dtype
        self.args = None

    def forward(self, x, *args, **kwargs):
        if isinstance(x, dict):
            return self.loss(x, *args, **kwargs)
        return self.predict(x, *args, **kwargs)

    def predict(self, x, profile=False, visualize=False, augment=False, embed=None, cuts=()):
        return self._predict_once(x, cuts)

    def _predict_once(self, x, cuts=()):
        """tasks.py:141-168 layer routing by m.f with the save list. `cuts` (layer indices) splits the autograd
        graph into backward stages for the DDP bucket overlap (engine/ddp.py): the tensors crossing each cut are
        replaced by detached leaves, recorded in self.stage_bounds."""
        first = 0
        layers = list(self.model)
        if x.dim() == 4 and x.shape[1] == 3:
            m0 = self.model[0]
            if self.compute_dtype == torch.bfloat16 and m0.f == -1 and getattr(m0, "stem_ok", lambda: False)():
                if getattr(self, "_uses", None) is None:
                    self._uses = consumer_counts(self.model)
                lazy = len(layers) > 1 and lazy_pair(m0, layers[1], self.save, cuts, self._uses)
                x = m0.forward_image(x, lazy=lazy)  # stem conv straight from the fp32 image (no NHWC copy of it)
                first = 1
            else:
                x = K.image_to_nhwc(x, self.compute_dtype, cpad=8)
        y = [x if self.model[0].i in self.save else None] if first else []
        if cuts and first and 0 in cuts:
            raise RuntimeError("stage cut after the fused stem layer is not supported")
        if getattr(self, "_uses", None) is None:
            self._uses = consumer_counts(self.model)
        try:
            x, bounds = route_layers(layers, self.save, x, y, first, cuts, self._uses)
        except BaseException:
            K.bnf_drop()  # a failed forward: its pending BN-act outputs must not be written into a later one
            raise
        K.bnf_clear()  # (every lazy BN-act output has been consumed; nothing may stay unwritten)
        if cuts:
            self.stage_bounds = bounds
        return x

    def loss(self, batch, preds=None, cuts=()):
        if getattr(self, "criterion", None) is None:
            self.criterion = self.init_criterion()
        preds = self.predict(batch["img"], cuts=cuts) if preds is None else preds
        return self.criterion(preds, batch)

    def init_criterion(self):
        from ..utils.loss import v8DetectionLoss
        return v8DetectionLoss(self)
