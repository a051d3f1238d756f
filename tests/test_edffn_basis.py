"""CPU check: the EDFFN patch filter restated as per-channel 64x64 operators (basis built with numpy fp64)
equals torch.fft.irfft2(rfft2(x) * w) as the reference computes it (block.py:2407-2409)."""
import numpy as np
import torch


def _basis():
    ps, nv = 8, 5
    eye = np.eye(64).reshape(64, 8, 8)
    spec = np.fft.rfft2(eye)
    B = np.empty((40, 64, 64))
    for u in range(8):
        for v in range(nv):
            f = np.zeros((8, nv))
            f[u, v] = 1
            B[u * nv + v] = np.fft.irfft2(spec * f, s=(8, 8)).reshape(64, 64).T
    return B


def test_basis_matches_torch_fft():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 8, 8, generator=g, dtype=torch.float64)
    w = 1 + 0.3 * torch.randn(4, 8, 5, generator=g, dtype=torch.float64)
    ref = torch.fft.irfft2(torch.fft.rfft2(x) * w, s=(8, 8))
    B = torch.from_numpy(_basis())
    M = torch.einsum("cu,uij->cij", w.reshape(4, 40), B)
    mine = torch.einsum("cij,cj->ci", M, x.reshape(4, 64)).reshape(4, 8, 8)
    assert torch.allclose(mine, ref, atol=1e-12), float((mine - ref).abs().max())
