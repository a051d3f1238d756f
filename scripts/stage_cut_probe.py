"""Which DDP stage cuts does the staged backward accept? python scripts/stage_cut_probe.py (GPU, bs 4 @320)."""
import sys
import traceback
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.engine.trainer import FusedTrainer  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

dev = torch.device("cuda", 0)
for cuts in [(6, 10), (7,), (10,), (20,), (11,), (13,), (19,), (21,), (7, 10, 20), (5,), (8,), (9,)]:
    model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"),
                           compute_dtype=torch.bfloat16).to(dev)
    tr = FusedTrainer(model, batch_size=4, stages=cuts)
    batch, _ = train_batch(4, 320, seed=0, device=dev)
    try:
        for _ in range(2):
            tr.step(batch)
        torch.cuda.synchronize()
        print(cuts, "ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print(cuts, "FAIL", type(e).__name__, str(e)[:100], flush=True)
        tb = traceback.format_exc().splitlines()
        print("   ", " | ".join(l.strip() for l in tb[-8:-1])[:600], flush=True)
