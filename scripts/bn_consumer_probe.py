"""How many training BatchNorm-act outputs feed a conv directly (the tensor object itself, no view / concat), and
how many of those convs are 1x1 stride-1 (the streaming kernel's shapes): the candidates for computing the BN
backward statistics in that conv's data-gradient epilogue. GPU, one eager step of the n model at bs 8, 320."""
import sys
from collections import Counter
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
import adrefine.kernels as K  # noqa: E402
from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.engine.trainer import FusedTrainer  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

cnt = Counter()
outs = {}
orig_bn = K.BNActFn.forward
orig_cv = K.Conv2dFn.forward


def bn_fwd(ctx, y, *a, **k):
    z = orig_bn(ctx, y, *a, **k)
    outs[id(z)] = z
    cnt["bn_outputs"] += 1
    return z


def cv_fwd(ctx, x, w, b, stride, pad, *a, **k):
    if id(x) in outs and outs[id(x)] is x:
        cnt["conv_direct"] += 1
        if w.shape[2] == w.shape[3] == 1 and (stride in (1, (1, 1))):
            cnt["conv_direct_1x1"] += 1
    cnt["convs"] += 1
    return orig_cv(ctx, x, w, b, stride, pad, *a, **k)


K.BNActFn.forward = staticmethod(bn_fwd)
K.Conv2dFn.forward = staticmethod(cv_fwd)
dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=8)
batch, _ = train_batch(8, 320, seed=0, device=dev)
tr.step(batch)
torch.cuda.synchronize()
print(dict(cnt))
