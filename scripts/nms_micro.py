"""adr_nms timing on real detector outputs (random-init YOLO-AD-Refine-n, bs 32, 640^2) at the predictor's and the
validator's settings, plus candidate statistics. Dev tool: run under rocprofv3 --kernel-trace --stats for the
per-kernel split. usage: python scripts/nms_micro.py [iters]"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

import torch  # noqa: E402

import adrefine.kernels as K  # noqa: E402
from adrefine.data.synthetic import images_u8  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402
from adrefine.utils.ops import non_max_suppression_padded  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    bs = int(os.environ.get("BS", 32))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = DetectionModel(str(ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"),
                           compute_dtype=torch.bfloat16).to(dev).eval()
    x = images_u8(bs, 640, seed=7).to(dev)
    packs = K.PackCache(cache_bn_coefs=True)
    with torch.no_grad(), K.pack_scope(packs):
        y = model(x)
    y = (y[0] if isinstance(y, (list, tuple)) else y).float().contiguous()
    sys.path.insert(1, str(ROOT))
    from oracle.recipe import synthetic_predictions  # dev script: synthetic head output of the NMS fixtures
    ys = synthetic_predictions(bs, 8400, 80, 640, seed=7).to(dev).contiguous()
    res = {"shape": list(y.shape), "mode": os.environ.get("ADR_NMS_MODE", "default"),
           "stop": os.environ.get("ADR_NMS_STOP", "0")}
    for name, conf, multi, y in (("predict", 0.25, False, y), ("val", 0.001, True, y),
                                 ("synth_predict", 0.25, False, ys), ("synth_val", 0.001, True, ys)):
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
        res[name] = {"us_per_call": round(1e3 * e0.elapsed_time(e1) / iters, 2), "candidates": cand,
                     "detections": int(n.sum()), "checksum": float(out.double().sum())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
