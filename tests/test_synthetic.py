"""The bench's synthetic stream (adrefine.data.synthetic) is the oracle's recipe (oracle/recipe.py)."""
import torch

from adrefine.data import synthetic as S
from oracle import recipe as R


def test_synthetic_stream_matches_oracle_recipe():
    assert torch.equal(S.images(2, 64, seed=5), R.synthetic_images(2, 64, seed=5))
    a, b = S.labels(16, 80, seed=9), R.synthetic_labels(16, 80, seed=9)
    for k in ("batch_idx", "cls", "bboxes"):
        assert torch.equal(a[k], b[k]), k
    assert a["bboxes"].min() >= 0 and (a["bboxes"][:, :2] + a["bboxes"][:, 2:] / 2).max() <= 1 + 1e-6
