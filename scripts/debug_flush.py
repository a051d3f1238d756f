"""One eager bs64 bf16 train step with ADR_DEBUG_BNSTAT=1: prints every BSTAT hand-off miss and every deferral
flush forced by a repeated gradient destination (with the call site). usage: ADR_DEBUG_BNSTAT=1 python ... (GPU)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402

from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.engine.trainer import FusedTrainer  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=64)
batch, _ = train_batch(64, 640, seed=0, device=dev)
tr.step(batch)
torch.cuda.synchronize()
print("=== second step ===", flush=True)
tr.step(batch)
torch.cuda.synchronize()
