"""Generate golden fixtures by importing the REFERENCE (read-only, /root/reference) — build container only.

Run:  python oracle/gen_golden.py            (refuses to run if /root/reference is missing)

The reference is imported with the stand-ins under oracle/stubs/ for packages absent from the image
(cv2, torchvision, timm, efficientnet_pytorch, mmcv). Two of those stand-ins carry arithmetic that the
reference calls on the hot path — torchvision.ops.nms and mmcv.ops.ModulatedDeformConv2d — and are restated
from their published algorithms (see the stub docstrings); fixtures that pass through them are marked
`unpinned_3rdparty` in tests/golden/MANIFEST.json.

Outputs (tests/golden/*.npz, small): per-module input/output/grad tuples at real channel counts, whole-net
eval outputs at 320^2 and 640^2 (bs 1), a train-mode step at 320^2 bs 2 (head outputs, loss, loss items,
per-parameter gradient norms), NMS outputs on synthetic predictions, and the state_dict manifests.
Weights come from oracle/recipe.py, so fixtures never store parameters.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
REPO = Path(__file__).resolve().parents[1]
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO / "oracle"))
from recipe import (recipe_state_dict, seeded_randn, synthetic_images,  # noqa: E402
                    synthetic_labels, synthetic_predictions)


def _import_reference():
    if not REF.is_dir():
        raise SystemExit("gen_golden: /root/reference is not present — fixtures are generated in the build container")
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    os.environ.setdefault("YOLO_CONFIG_DIR", "/tmp/adr_yolo_cfg")
    sys.path.insert(0, str(REPO / "oracle" / "stubs"))
    sys.path.insert(1, str(REF))
    import ultralytics  # noqa: F401
    from ultralytics.nn import tasks
    from ultralytics.nn.modules import block, conv, head
    from ultralytics.utils import loss as uloss
    from ultralytics.utils import ops as uops
    return tasks, block, conv, head, uloss, uops


def _np(t):
    return t.detach().cpu().numpy()


def load_recipe(module):
    sd = module.state_dict()
    rec = recipe_state_dict([(k, v.shape) for k, v in sd.items()])
    module.load_state_dict(rec, strict=True)
    return rec


def module_fixture(name, mod, specs, seed, extra=None):
    """Run mod(*inputs) in train mode, backprop a seeded random upstream gradient, save in/out/grads."""
    torch.manual_seed(seed)
    load_recipe(mod)
    mod.train()
    specs = [sp if isinstance(sp, tuple) and isinstance(sp[0], tuple) else (tuple(sp), 11) for sp in specs]
    inputs = [seeded_randn(*shp, seed=sd) for shp, sd in specs]
    ins = [x.clone().requires_grad_(True) for x in inputs]
    out = mod(list(ins)) if getattr(mod, "_list_input", False) else mod(ins[0])  # Detect writes into its list
    outs = out if isinstance(out, (list, tuple)) else [out]
    g = torch.Generator().manual_seed(seed + 1)
    gouts = [torch.randn(o.shape, generator=g) for o in outs]
    torch.autograd.backward(list(outs), gouts)
    d = {f"in{i}_shape": np.array(x.shape) for i, x in enumerate(inputs)}
    d.update({f"in{i}_seed": np.array(sd) for i, (_, sd) in enumerate(specs)})
    d.update({f"out{i}": _np(o) for i, o in enumerate(outs)})
    d.update({f"gin{i}": _np(x.grad) for i, x in enumerate(ins)})
    gn = {k: float(p.grad.norm()) for k, p in mod.named_parameters() if p.grad is not None}
    d["param_grad_norms_keys"] = np.array(list(gn.keys()))
    d["param_grad_norms"] = np.array(list(gn.values()), dtype=np.float64)
    if extra:
        d.update(extra)
    np.savez_compressed(OUT / f"mod_{name}.npz", **d)
    return d


def main():
    tasks, block, conv, head, uloss, uops = _import_reference()
    OUT.mkdir(parents=True, exist_ok=True)
    torch.set_num_threads(8)
    only_nms = "--only-nms" in sys.argv
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
    if only:
        manifest = json.loads((OUT / "MANIFEST.json").read_text())

        def note(name, what, cites, unpinned=False):
            manifest["fixtures"][name] = {"what": what, "reference": cites, "unpinned_3rdparty": unpinned}
        for what in only[0].split(","):
            globals()[f"{what}_fixtures"](tasks, block, conv, head, uloss, uops, note)
        manifest.update(manifest_extra)
        (OUT / "MANIFEST.json").write_text(json.dumps(manifest, indent=1))
        return
    if only_nms:
        manifest = json.loads((OUT / "MANIFEST.json").read_text())
    else:
        manifest = {"generator": "oracle/gen_golden.py", "reference": "wcq99681-svg/YOLO-AD-Refine @ 2025-12-26",
                    "torch": torch.__version__, "fixtures": {}}

    def note(name, what, cites, unpinned=False):
        manifest["fixtures"][name] = {"what": what, "reference": cites, "unpinned_3rdparty": unpinned}

    if only_nms:
        nms_fixtures(uops, note)
        (OUT / "MANIFEST.json").write_text(json.dumps(manifest, indent=1))
        return

    # ---------------- per-module fixtures (train mode, bs 2, real channel counts, small spatial) ---------------
    m = conv.Conv(16, 32, 3, 2)
    for mm in m.modules():
        if isinstance(mm, torch.nn.BatchNorm2d):
            mm.eps, mm.momentum = 1e-3, 0.03
    module_fixture("conv_k3s2", m, [((2, 16, 24, 24), 11)], 21)
    note("mod_conv_k3s2", "Conv(16,32,3,2) train fwd/bwd", "nn/modules/conv.py:36-54")

    def bnfix(mod):
        for mm in mod.modules():
            if isinstance(mm, torch.nn.BatchNorm2d):
                mm.eps, mm.momentum = 1e-3, 0.03
        return mod

    module_fixture("c3k2", bnfix(block.C3k2(32, 64, 1, False, 0.25)), [((2, 32, 20, 20), 11)], 22)
    note("mod_c3k2", "C3k2(32,64,1,False,0.25)", "block.py:731-739,232-247,341-354")
    module_fixture("c3k2_mlca_c3k", bnfix(block.C3k2_MLCA(128, 128, 1, True)), [((2, 128, 20, 20), 11)], 23)
    note("mod_c3k2_mlca_c3k", "C3k2_MLCA(128,128,1,True)", "block.py:1540-1605")
    module_fixture("c3k2_mlca", bnfix(block.C3k2_MLCA(128, 128, 1, False)), [((2, 128, 20, 20), 12)], 24)
    note("mod_c3k2_mlca", "C3k2_MLCA(128,128,1,False) @20x20", "block.py:1540-1605")
    module_fixture("sppf", bnfix(block.SPPF(256, 256, 5)), [((2, 256, 10, 10), 11)], 25)
    note("mod_sppf", "SPPF(256,256,5)", "block.py:177-196")
    module_fixture("ela", block.ELA_HSFPN(128), [((2, 128, 20, 20), 11)], 26)
    note("mod_ela", "ELA_HSFPN(128, flag=True)", "block.py:1408-1424")
    module_fixture("ela_noflag", block.ELA_HSFPN(128, False), [((2, 128, 20, 20), 11)], 27)
    note("mod_ela_noflag", "ELA_HSFPN(128, flag=False)", "block.py:1408-1424")
    module_fixture("convT", torch.nn.ConvTranspose2d(128, 128, 3, 2, 1, 1), [((2, 128, 10, 10), 11)], 28)
    note("mod_convT", "nn.ConvTranspose2d(128,128,3,2,1,1)", "tasks.py:1005 (yaml L13/L20)")
    fu = block.Fusion([128, 128], "bifpn")
    fu._list_input = True
    module_fixture("fusion", fu, [((2, 128, 10, 10), 1), ((2, 128, 10, 10), 2)], 29)
    note("mod_fusion", "Fusion([128,128],'bifpn')", "block.py:1500-1537")
    module_fixture("c2ptssa", bnfix(block.C2PTSSA(256, 256, 1)), [((2, 256, 20, 20), 11)], 30)
    note("mod_c2ptssa", "C2PTSSA(256,256,1) @20x20 (MHA over 1200 tokens, EDFFN patch FFT)", "block.py:2376-2710")
    mona_m = bnfix(block.C2TSSA_DYT_Mona_EDFFN(256, 256, 1))
    for mm in mona_m.modules():
        if isinstance(mm, torch.nn.Dropout):
            mm.p = 0.0
    module_fixture("c2tssa_mona", mona_m, [((2, 256, 20, 20), 11)], 31)
    note("mod_c2tssa_mona", "C2TSSA_DYT_Mona_EDFFN(256,256,1) (dropout p=0)", "block.py:1624-1709, mona.py")
    hd = head.AYHead(80, [128, 128, 128])
    hd.stride = torch.tensor([8.0, 16.0, 32.0])
    for mm in hd.modules():
        if isinstance(mm, torch.nn.BatchNorm2d):
            mm.eps, mm.momentum = 1e-3, 0.03
    hd._list_input = True
    module_fixture("ayhead", hd, [((2, 128, 16, 16), 3), ((2, 128, 8, 8), 4), ((2, 128, 4, 4), 5)], 32)
    note("mod_ayhead", "AYHead(80,[128]*3) train fwd/bwd incl. DCNv2 (mmcv restated)", "head.py:1049-1252", True)

    # ---------------- whole network -----------------------------------------------------------------------------
    for tag, yaml_name in (("701", "yolo11-701-YOLO-AD-Refine.yaml"), ("697", "yolo11-697-newfpn+mona+AYHead+mlca3.yaml")):
        model = tasks.DetectionModel(str(REF / "z-yaml" / yaml_name), verbose=False)
        for mm in model.modules():
            if isinstance(mm, torch.nn.Dropout):
                mm.p = 0.0
        sd = model.state_dict()
        manifest[f"state_dict_{tag}"] = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]
        rec = load_recipe(model)
        model.args = type("H", (), {"box": 7.5, "cls": 0.5, "dfl": 1.5})()
        # eval outputs
        model.eval()
        sizes = (320, 640) if tag == "701" else (320,)
        for S in sizes:
            x = synthetic_images(1, S, seed=0)
            with torch.no_grad():
                y, outs = model(x)
            np.savez_compressed(OUT / f"net{tag}_eval_{S}.npz", img_seed=np.array(0), y=_np(y))
            note(f"net{tag}_eval_{S}", f"{yaml_name} eval forward bs1 {S}^2 (recipe weights)",
                 "nn/tasks.py:141-168, head.py:1181-1204", True)
        # train step at 320, bs 2
        model.load_state_dict(rec, strict=True)
        model.train()
        x = synthetic_images(2, 320, seed=0)
        batch = synthetic_labels(2, 80, seed=1)
        preds = model(x)
        crit = uloss.v8DetectionLoss(model)
        loss, items = crit(preds, batch)
        for p in preds:
            p.retain_grad()
        loss.backward()
        gn = {k: float(p.grad.norm()) if p.grad is not None else 0.0 for k, p in model.named_parameters()}
        bn_rm = {k: _np(v) for k, v in model.state_dict().items() if k in
                 ("model.0.bn.running_mean", "model.0.bn.running_var", "model.33.coord_attention_reg.bn1.running_var")}
        d = {"img_seed": np.array(0), "batch_idx": _np(batch["batch_idx"]), "cls": _np(batch["cls"]), "bboxes": _np(batch["bboxes"]),
             "loss": _np(loss), "items": _np(items), "gn_keys": np.array(list(gn.keys())),
             "gn": np.array(list(gn.values()), dtype=np.float64)}
        for i, p in enumerate(preds):
            d[f"pred{i}"] = _np(p)
            d[f"gpred{i}_norm"] = np.array(float(p.grad.norm()))
            d[f"gpred{i}_sum"] = np.array(float(p.grad.sum()))
        for k, v in bn_rm.items():
            d["post_" + k] = v
        np.savez_compressed(OUT / f"net{tag}_train_320.npz", **d)
        note(f"net{tag}_train_320", f"{yaml_name} train fwd + v8DetectionLoss + bwd, bs2 320^2",
             "engine/trainer.py:383-393, utils/loss.py:419-520, utils/tal.py:39-265", True)

    # ---------------- loss on fixed head outputs (independent of the network) ----------------------------------
    hd2 = head.AYHead(80, [128, 128, 128])
    hd2.stride = torch.tensor([8.0, 16.0, 32.0])

    class _M(torch.nn.Module):
        def __init__(s):
            super().__init__()
            s.model = torch.nn.ModuleList([hd2])
            s.args = type("H", (), {"box": 7.5, "cls": 0.5, "dfl": 1.5})()

    crit = uloss.v8DetectionLoss(_M())
    for S, bs, seed in ((640, 4, 41), (320, 4, 42)):
        g = torch.Generator().manual_seed(seed)
        feats = [torch.randn(bs, 144, S // s, S // s, generator=g) for s in (8, 16, 32)]
        for f in feats:
            f[:, :64] *= 2.0
            f.requires_grad_(True)
        batch = synthetic_labels(bs, 80, seed=seed + 1)
        loss, items = crit(feats, batch)
        loss.backward()
        d = {"batch_idx": _np(batch["batch_idx"]), "cls": _np(batch["cls"]), "bboxes": _np(batch["bboxes"]),
             "loss": _np(loss), "items": _np(items)}
        for i, f in enumerate(feats):
            d[f"feat{i}_seed"] = np.array([seed, i])
            d[f"gfeat{i}"] = _np(f.grad).astype(np.float32) if S == 320 else np.zeros(0, np.float32)
            d[f"gfeat{i}_norm"] = np.array(float(f.grad.norm()))
        np.savez_compressed(OUT / f"loss_{S}_bs{bs}.npz", **d)
        note(f"loss_{S}_bs{bs}", "v8DetectionLoss on seeded randn head outputs (x2 on box channels)",
             "utils/loss.py:419-520, tal.py:39-265, metrics.py:74-125,539-564")

    nms_fixtures(uops, note)

    (OUT / "MANIFEST.json").write_text(json.dumps(manifest, indent=1))
    print("wrote", len(list(OUT.glob("*.npz"))), "fixtures to", OUT)


def _hyp():
    return type("H", (), {"box": 7.5, "cls": 0.5, "dfl": 1.5})()


def _eval_fixture(model, S, name):
    model.eval()
    x = synthetic_images(1, S, seed=0)
    with torch.no_grad():
        y, _ = model(x)
    np.savez_compressed(OUT / f"{name}.npz", img_seed=np.array(0), y=_np(y))


def _train_fixture(model, uloss, S, bs, name, rec):
    """Train-mode forward + v8DetectionLoss + backward at S^2, batch bs (recipe weights reloaded first)."""
    model.load_state_dict(rec, strict=True)
    model.train()
    x = synthetic_images(bs, S, seed=0)
    batch = synthetic_labels(bs, 80, seed=1)
    preds = model(x)
    crit = uloss.v8DetectionLoss(model)
    loss, items = crit(preds, batch)
    for p in preds:
        p.retain_grad()
    loss.backward()
    gn = {k: float(p.grad.norm()) if p.grad is not None else 0.0 for k, p in model.named_parameters()}
    d = {"img_seed": np.array(0), "img_size": np.array(S), "batch_idx": _np(batch["batch_idx"]),
         "cls": _np(batch["cls"]), "bboxes": _np(batch["bboxes"]), "loss": _np(loss), "items": _np(items),
         "gn_keys": np.array(list(gn.keys())), "gn": np.array(list(gn.values()), dtype=np.float64)}
    for i, p in enumerate(preds):
        d[f"pred{i}"] = _np(p)
        d[f"gpred{i}_norm"] = np.array(float(p.grad.norm()))
        d[f"gpred{i}_sum"] = np.array(float(p.grad.sum()))
    sd = model.state_dict()
    d["post_model.0.bn.running_mean"] = _np(sd["model.0.bn.running_mean"])
    d["post_model.0.bn.running_var"] = _np(sd["model.0.bn.running_var"])
    np.savez_compressed(OUT / f"{name}.npz", **d)


def yolo11_fixtures(tasks, block, conv, head, uloss, uops, note):
    """Config 1: the stock yolo11n (tests/configs/yolo11.yaml, scale n) — construction facts of the reference's
    DetectionModel (probe strides, bias_init, the probe's BatchNorm side effects), eval 320/640, a train step at
    320 bs2, and module fixtures for C2PSA and Detect."""
    global manifest_extra
    torch.manual_seed(0)
    model = tasks.DetectionModel(str(REPO / "tests" / "configs" / "yolo11n.yaml"), verbose=False)
    m = model.model[-1]
    sd = model.state_dict()
    manifest_extra["state_dict_y11n"] = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]
    init = {"stride": _np(m.stride), "cv2_bias": np.stack([_np(a[-1].bias) for a in m.cv2]),
            "cv3_bias": np.stack([_np(b[-1].bias) for b in m.cv3]),
            "bn_running_var": np.concatenate([_np(v).ravel() for k, v in sd.items() if k.endswith("running_var")]),
            "bn_running_mean": np.concatenate([_np(v).ravel() for k, v in sd.items() if k.endswith("running_mean")]),
            "bn_nbt": np.array([int(v) for k, v in sd.items() if k.endswith("num_batches_tracked")]),
            "bn_eps": np.array([mm.eps for mm in model.modules() if isinstance(mm, torch.nn.BatchNorm2d)]),
            "bn_momentum": np.array([mm.momentum for mm in model.modules() if isinstance(mm, torch.nn.BatchNorm2d)]),
            "n_params": np.array(sum(p.numel() for p in model.parameters()))}
    np.savez_compressed(OUT / "y11n_init.npz", **init)
    note("y11n_init", "yolo11n DetectionModel construction: probe strides, Detect.bias_init, BN state after the "
         "zero-image probe, BN eps/momentum after initialize_weights", "nn/tasks.py:309-350, head.py:137-147")
    rec = load_recipe(model)
    model.args = _hyp()
    for S in (320, 640):
        _eval_fixture(model, S, f"y11n_eval_{S}")
        note(f"y11n_eval_{S}", f"yolo11n eval forward bs1 {S}^2 (recipe weights)", "nn/tasks.py:141-168, head.py:55-115")
    _train_fixture(model, uloss, 320, 2, "y11n_train_320", rec)
    note("y11n_train_320", "yolo11n train fwd + v8DetectionLoss + bwd, bs2 320^2",
         "engine/trainer.py:383-393, utils/loss.py:419-520, utils/tal.py:39-265")

    def bnfix(mod):
        for mm in mod.modules():
            if isinstance(mm, torch.nn.BatchNorm2d):
                mm.eps, mm.momentum = 1e-3, 0.03
        return mod
    module_fixture("c2psa", bnfix(block.C2PSA(256, 256, 1)), [((2, 256, 20, 20), 11)], 33)
    note("mod_c2psa", "C2PSA(256,256,1) @20x20 (2 heads, key_dim 32)", "block.py:874-1045")
    module_fixture("c2psa_l", bnfix(block.C2PSA(512, 512, 2)), [((2, 512, 10, 10), 12)], 34)
    note("mod_c2psa_l", "C2PSA(512,512,2) @10x10 (4 heads, 2 blocks)", "block.py:874-1045")
    dt = bnfix(head.Detect(80, [64, 128, 256]))
    dt.stride = torch.tensor([8.0, 16.0, 32.0])
    dt._list_input = True
    module_fixture("detect", dt, [((2, 64, 16, 16), 3), ((2, 128, 8, 8), 4), ((2, 256, 4, 4), 5)], 35)
    note("mod_detect", "Detect(80,[64,128,256]) train fwd/bwd", "head.py:21-70")


def lscale_fixtures(tasks, block, conv, head, uloss, uops, note):
    """Config 5 groundwork: the 701 yaml at scale 'l' (C3k2 c3k=True per tasks.py:1050-1051, C2PTSSA c=256 with 4
    heads, AYHead hidc 512), eval 256^2 bs1 and a train step at 256^2 bs2 (CPU-sized stand-ins for 1280^2)."""
    import yaml as _yaml
    global manifest_extra
    d = _yaml.safe_load((REF / "z-yaml" / "yolo11-701-YOLO-AD-Refine.yaml").read_text())
    d["scale"] = "l"
    model = tasks.DetectionModel(d, verbose=False)
    for mm in model.modules():
        if isinstance(mm, torch.nn.Dropout):
            mm.p = 0.0
    sd = model.state_dict()
    manifest_extra["state_dict_701l"] = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]
    rec = load_recipe(model)
    model.args = _hyp()
    _eval_fixture(model, 256, "net701l_eval_256")
    note("net701l_eval_256", "701 yaml scale l eval forward bs1 256^2 (recipe weights)",
         "nn/tasks.py:141-168,1050-1051, head.py:1181-1204", True)
    _train_fixture(model, uloss, 256, 2, "net701l_train_256", rec)
    note("net701l_train_256", "701 yaml scale l train fwd + v8DetectionLoss + bwd, bs2 256^2",
         "engine/trainer.py:383-393, utils/loss.py:419-520", True)


manifest_extra = {}

# parameters whose FULL gradient tensor the 701 train-step fixture keeps (one or more per module family on the
# path: stem Conv-BN, C3k2_MLCA, C3k bottleneck, C2PTSSA attention / EDFFN, ELA, BiFPN Fusion, nn.Conv2d rows,
# AYHead stems / shared Conv_GN / DyDCNv2 / CoordAtt BN / output convs / Scale)
GRAD_KEYS = ("model.0.conv.weight", "model.0.bn.weight", "model.0.bn.bias", "model.6.cv2.conv.weight",
             "model.6.cv2.bn.weight", "model.8.m.0.cv1.conv.weight", "model.10.m.0.attn.qkv_projections.0.weight",
             "model.10.m.0.attn.cross_scale_fusion.in_proj_weight", "model.10.m.0.ffn.project_in.weight",
             "model.12.weight", "model.28.fusion_weight", "model.33.stems.0.conv.weight",
             "model.33.share_conv.0.conv.weight", "model.33.share_conv.0.gn.weight", "model.33.DyDCNV2.conv.weight",
             "model.33.coord_attention_reg.bn1.weight", "model.33.cv2.weight", "model.33.cv2.bias",
             "model.33.cv3.weight", "model.33.cv3.bias", "model.33.scale.0.scale")


def grads_fixtures(tasks, block, conv, head, uloss, uops, note):
    """Elementwise parameter-gradient parity: the reference's 701 train step at 320^2 bs 2 (the inputs, labels and
    recipe weights of net701_train_320) with the full dL/dtheta tensors of GRAD_KEYS (nn/tasks.py:290-302 loss ->
    autograd backward; utils/loss.py:419-520)."""
    model = tasks.DetectionModel(str(REF / "z-yaml" / "yolo11-701-YOLO-AD-Refine.yaml"), verbose=False)
    rec = load_recipe(model)
    model.args = _hyp()
    model.load_state_dict(rec, strict=True)
    model.train()
    x = synthetic_images(2, 320, seed=0)
    batch = synthetic_labels(2, 80, seed=1)
    preds = model(x)
    loss, items = uloss.v8DetectionLoss(model)(preds, batch)
    loss.backward()
    P = dict(model.named_parameters())
    d = {"img_seed": np.array(0), "img_size": np.array(320), "batch_idx": _np(batch["batch_idx"]),
         "cls": _np(batch["cls"]), "bboxes": _np(batch["bboxes"]), "loss": _np(loss), "items": _np(items),
         "keys": np.array(GRAD_KEYS)}
    for i, k in enumerate(GRAD_KEYS):
        d[f"g{i}"] = _np(P[k].grad).astype(np.float32)
    np.savez_compressed(OUT / "net701_grads_320.npz", **d)
    note("net701_grads_320", "701 train step bs2 320^2: full parameter gradients of a subset (GRAD_KEYS)",
         "nn/tasks.py:290-302, utils/loss.py:419-520, head.py:1049-1252", True)


def metrics_fixtures(tasks, block, conv, head, uloss, uops, note):
    """Validator metrics tail on synthetic detections: per-image box_iou (utils/metrics.py:52) + greedy
    match_predictions (engine/validator.py:221) -> tp (N, 10); ap_per_class (metrics.py:1144) + Metric
    mean_results / fitness (metrics.py:1340-1358). Inputs are stored in the fixture."""
    from ultralytics.engine.validator import BaseValidator
    from ultralytics.utils import metrics as M
    rng = np.random.default_rng(123)
    preds, labels = [], []
    for img in range(6):
        n = int(rng.integers(0 if img == 5 else 2, 14))
        xy = rng.uniform(20, 560, (n, 2))
        wh = rng.uniform(8, 200, (n, 2))
        gt = np.concatenate([xy, np.minimum(xy + wh, 639)], 1)
        gcls = rng.integers(0, 12, n).astype(np.float32)
        rows = []
        for k in range(n):
            if rng.random() < 0.8:  # a detection of this object, jittered
                j = gt[k] + rng.normal(0, 0.08, 4) * np.r_[wh[k], wh[k]]
                c = gcls[k] if rng.random() < 0.9 else float(rng.integers(0, 12))
                rows.append([*j, rng.uniform(0.2, 1.0), c])
        for _ in range(int(rng.integers(0, 20))):  # false positives
            xy0 = rng.uniform(0, 600, 2)
            rows.append([*xy0, *(xy0 + rng.uniform(5, 150, 2)), rng.uniform(0.001, 0.7), float(rng.integers(0, 12))])
        if img == 4:
            rows = []  # an image with labels and no detections
        pr = np.array(rows, dtype=np.float32).reshape(-1, 6)
        preds.append(pr)
        labels.append(np.concatenate([np.full((n, 1), img, np.float32), gcls[:, None], gt.astype(np.float32)], 1))
    v = BaseValidator.__new__(BaseValidator)
    v.iouv = torch.linspace(0.5, 0.95, 10)
    tps, confs, pcls, tcls = [], [], [], []
    for img, (pr, lb) in enumerate(zip(preds, labels)):
        p = torch.from_numpy(pr)
        if len(lb) and len(pr):
            iou = M.box_iou(torch.from_numpy(lb[:, 2:6]), p[:, :4])
            tp = v.match_predictions(p[:, 5], torch.from_numpy(lb[:, 1]), iou).numpy()
        else:
            tp = np.zeros((len(pr), 10), dtype=bool)
        tps.append(tp)
        confs.append(pr[:, 4])
        pcls.append(pr[:, 5])
        tcls.append(lb[:, 1])
    tp, conf, pc, tc = (np.concatenate(a, 0) for a in (tps, confs, pcls, tcls))
    res = M.ap_per_class(tp, conf, pc, tc)
    met = M.Metric()
    met.update(res[2:])
    d = {"preds": np.concatenate([np.concatenate([np.full((len(p), 1), i, np.float32), p], 1)
                                  for i, p in enumerate(preds)], 0),
         "labels": np.concatenate(labels, 0), "tp": tp, "p": res[2], "r": res[3], "ap": res[5],
         "ap_class_index": res[6], "mean_results": np.array(met.mean_results(), dtype=np.float64),
         "fitness": np.array(met.fitness(), dtype=np.float64)}
    np.savez_compressed(OUT / "metrics_val.npz", **d)
    note("metrics_val", "validator TP matching + ap_per_class + Metric on synthetic detections (6 images)",
         "models/yolo/detect/val.py:125-229, engine/validator.py:221-261, utils/metrics.py:52,1112-1360")


def augment_fixtures(tasks, block, conv, head, uloss, uops, note):
    """Training augmentation chain (data/augment.py v8_transforms :2273-2335 + Format :1920-2100, collated by
    YOLODataset.collate_fn, data/dataset.py:230-246) on synthetic items (recipe.synthetic_aug_items), the python /
    numpy RNGs seeded, through the reference's own transform code. The OpenCV calls in it (RandomHSV cvtColor / LUT,
    RandomPerspective warpAffine / getRotationMatrix2D) run on oracle/stubs/cv2 (restated, unpinned)."""
    import random
    from types import SimpleNamespace

    from recipe import AUG_HYPS, synthetic_aug_items
    from ultralytics.data.augment import Format, v8_transforms
    from ultralytics.data.dataset import YOLODataset
    from ultralytics.utils.instance import Instances

    class _DS:
        def __init__(self, items, imgsz):
            self.items, self.imgsz = items, imgsz
            self.buffer = list(range(len(items)))
            self.data = {"flip_idx": []}
            self.use_keypoints = False

        def __len__(self):
            return len(self.items)

        def get_image_and_label(self, i):
            it = self.items[i]
            h, w = it["img"].shape[:2]
            return {"im_file": f"syn{i}.jpg", "ori_shape": (h, w), "resized_shape": (h, w), "ratio_pad": (1.0, 1.0),
                    "img": it["img"].copy(), "cls": it["cls"].copy(),
                    "instances": Instances(it["bboxes"].copy(), np.zeros((0, 1000, 2), dtype=np.float32), None,
                                           bbox_format="xywh", normalized=True)}

    for name, imgsz, seed, order in (("aug_default_256", 256, 5, [0, 1, 2, 3]),
                                     ("aug_rot_256", 256, 9, [4, 5, 6, 7, 0, 2])):
        hyp = SimpleNamespace(**AUG_HYPS[name.split("_")[1]])
        ds = _DS(synthetic_aug_items(8, imgsz), imgsz)
        T = v8_transforms(ds, imgsz, hyp)
        T.append(Format(bbox_format="xywh", normalize=True, return_mask=False, return_keypoint=False,
                        return_obb=False, batch_idx=True, mask_ratio=4, mask_overlap=True, bgr=hyp.bgr))
        random.seed(seed)
        np.random.seed(seed)
        batch = YOLODataset.collate_fn([T(ds.get_image_and_label(i)) for i in order])
        np.savez_compressed(OUT / f"{name}.npz", img=_np(batch["img"]), cls=_np(batch["cls"]),
                            bboxes=_np(batch["bboxes"]), batch_idx=_np(batch["batch_idx"]), seed=seed, imgsz=imgsz,
                            order=np.array(order))
        note(name, f"v8_transforms + Format + collate_fn, hyp {name.split('_')[1]}, imgsz {imgsz}, items {order}",
             ["data/augment.py:489-865", "data/augment.py:951-1298", "data/augment.py:1301-1473",
              "data/augment.py:1920-2100", "data/augment.py:2273-2335", "data/dataset.py:230-246"], unpinned=True)
        print(name, batch["img"].shape, batch["bboxes"].shape)


def nms_fixtures(uops, note):
    """utils/ops.py:163-312 on the exactly-reproducible synthetic predictions (recipe.synthetic_predictions)."""
    pred = synthetic_predictions(2, 8400, 80, 640, seed=7)
    for name, conf, iou, ml in (("predict", 0.25, 0.7, False), ("val", 0.001, 0.7, True), ("tight", 0.25, 0.45, False)):
        # max_time_img raised so the reference's wall-clock cut-off (ops.py:234, 308-310) cannot truncate the
        # fixture when it runs over the slow Python NMS stand-in
        out = uops.non_max_suppression(pred.clone(), conf, iou, multi_label=ml, max_det=300, max_time_img=1e4)
        d = {f"out{i}": _np(o) for i, o in enumerate(out)}
        d["conf"], d["iou"], d["multi_label"] = np.array(conf), np.array(iou), np.array(ml)
        np.savez_compressed(OUT / f"nms_{name}.npz", **d)
        note(f"nms_{name}", f"non_max_suppression(conf={conf}, iou={iou}, multi_label={ml}) on seed-7 predictions",
             "utils/ops.py:163-312 -> torchvision.ops.nms (restated)", True)


if __name__ == "__main__":
    main()
