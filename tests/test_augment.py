"""Training augmentation chain (reference data/augment.py v8_transforms :2273-2335 + Format + collate_fn) against
fixtures made by running the reference's own transform code (oracle/gen_golden.py `augment`; its OpenCV calls on
the numpy restatement in oracle/stubs/cv2, so OpenCV's internals are PARITY UNPINNED, the reference's RNG order,
matrices and label arithmetic are pinned).

CPU: the host side of adrefine.data.augment (draws, boxes, classes, the image plans) — boxes and classes
bit-exact; each plan, materialised by the numpy executor in tests/aug_util.py, equals the fixture image exactly.
GPU: adr_augment_u8 renders the same plans into the collated uint8 batch bit-exactly (all stages fused, one
launch)."""
from pathlib import Path

import numpy as np
import pytest
import torch

from aug_util import CONFIGS, execute_plan, run_chain

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("name", list(CONFIGS))
def test_augment_labels_and_plans_vs_reference(name):
    g = np.load(GOLD / f"{name}.npz", allow_pickle=False)
    out = run_chain(name)
    cls = torch.cat([o["cls"] for o in out]).numpy()
    bboxes = torch.cat([o["bboxes"] for o in out]).numpy()
    bidx = torch.cat([o["batch_idx"] + i for i, o in enumerate(out)]).numpy()
    assert np.array_equal(cls, g["cls"]) and np.array_equal(bidx, g["batch_idx"])
    assert bboxes.dtype == g["bboxes"].dtype and np.array_equal(bboxes, g["bboxes"])
    for i, o in enumerate(out):
        img = execute_plan(o["img"])
        diff = int((img.astype(np.int32) - g["img"][i].astype(np.int32)).__abs__().max())
        assert img.shape == g["img"][i].shape and diff == 0, (i, diff)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CONFIGS))
def test_augment_gpu_render_vs_reference(name):
    from adrefine.data.augment import collate_fn
    g = np.load(GOLD / f"{name}.npz", allow_pickle=False)
    batch = collate_fn(run_chain(name))
    torch.cuda.synchronize()
    img = batch["img"].cpu().numpy()
    assert img.dtype == np.uint8 and img.shape == g["img"].shape
    bad = np.argwhere(img != g["img"])
    assert len(bad) == 0, (len(bad), bad[:5].tolist())
    assert np.array_equal(batch["bboxes"].numpy(), g["bboxes"]) and np.array_equal(batch["cls"].numpy(), g["cls"])
    assert np.array_equal(batch["batch_idx"].numpy(), g["batch_idx"])
