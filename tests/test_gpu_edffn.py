"""EDFFN spectral patch filter (reference nn/modules/block.py:2399-2413: reflect-pad to a multiple of 8, per-patch
rfft2 * fft -> irfft2, crop) on bf16 tensors: the matrix-core apply (adr_c2p.hip edffn_apply_mfma_kernel, fp32 MFMA)
against the per-channel scalar kernel (ADR_EDFFN_MFMA=0) and a torch fp64 restatement of the same per-channel 64x64
operators. Forward output, input gradient and the fft-weight gradient. The fp32 parity path (reference fixtures,
test_gpu_blocks.py) keeps the scalar kernel."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, M):
    """y[n, c, patch pos i] = sum_j M[c][i][j] xpad[n, c, patch pos j] in fp64, cropped (x: N C H W float)."""
    N, C, H, W = x.shape
    Hp, Wp = (H + 7) // 8 * 8, (W + 7) // 8 * 8
    xp = F.pad(x.double(), (0, Wp - W, 0, Hp - H), mode="reflect")
    pt = xp.view(N, C, Hp // 8, 8, Wp // 8, 8).permute(0, 1, 2, 4, 3, 5).reshape(N, C, Hp // 8, Wp // 8, 64)
    yp = torch.einsum("cij,nchwj->nchwi", M.double(), pt)
    y = yp.view(N, C, Hp // 8, Wp // 8, 8, 8).permute(0, 1, 2, 4, 3, 5).reshape(N, C, Hp, Wp)
    return y[:, :, :H, :W]


@pytest.mark.parametrize("N,C,H,W", [(64, 128, 20, 20), (3, 64, 13, 20)])
def test_edffn_mfma_matches_scalar_and_fp64(N, C, H, W, monkeypatch):
    from adrefine import kernels as K
    torch.manual_seed(0)
    x0 = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fft = torch.randn(C, 8, 5, device="cuda") * 0.5
    gy = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("ADR_EDFFN_MFMA", mode)
        x = x0.clone().requires_grad_(True)
        f = fft.clone().requires_grad_(True)
        y = K.edffn_filter(x, f)
        y.backward(gy)
        out[mode] = (y.detach().float(), x.grad.float(), f.grad.float())
    basis = K.edffn_basis(x0.device)
    M = torch.einsum("cu,uij->cij", fft.view(C, -1), basis)
    yref = _ref(x0.float(), M)
    scale = float(yref.abs().max())
    for mode in ("0", "1"):
        err = float((out[mode][0] - yref).abs().max())
        assert err <= scale * 2 ** -7, (mode, err, scale)
    # same fp32 sums in another order: the bf16 outputs agree to one rounding
    assert float((out["1"][0] - out["0"][0]).abs().max()) <= scale * 2 ** -7
    gs = float(out["0"][1].abs().max())
    assert float((out["1"][1] - out["0"][1]).abs().max()) <= gs * 2 ** -7
    fr = out["0"][2]
    assert float((out["1"][2] - fr).norm() / fr.norm()) < 1e-4
