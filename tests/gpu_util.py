"""Helpers for GPU parity tests: run an adrefine module on cuda:0 and the CPU oracle on the same seeded
inputs / recipe weights, then compare outputs, input gradients and parameter gradients."""
import numpy as np
import torch

from recipe import recipe_state_dict

# fp32 parity mode: elementwise; bf16 mode: bf16 storage of every activation (8 mantissa bits) compounds
# through deep chains, so bf16 checks use a loose elementwise bound plus a relative-L2 bound.
TOL = {torch.float32: dict(rtol=2e-4, atol=2e-4), torch.bfloat16: dict(rtol=1.5e-1, atol=5e-2, l2=6e-2)}


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def assert_close(a, b, rtol, atol, what="", l2=None):
    """max|a-b| <= atol + rtol*max|b|; with l2 set (bf16 checks) also ||a-b|| / ||b|| <= l2."""
    a = a.detach().double().cpu()
    b = torch.as_tensor(np.asarray(b)).double() if not torch.is_tensor(b) else b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = float((a - b).abs().max()) if a.numel() else 0.0
    scale = float(b.abs().max()) if b.numel() else 0.0
    assert err <= atol + rtol * scale, f"{what}: max|d|={err:.3e} scale={scale:.3e}"
    if l2 is not None and a.numel():
        rel = float((a - b).norm() / (b.norm() + 1e-30))
        assert rel <= l2, f"{what}: rel L2 {rel:.3e} > {l2}"


def load_recipe_into(module):
    sd = module.state_dict()
    rec = recipe_state_dict([(k, v.shape) for k, v in sd.items()])
    module.load_state_dict(rec, strict=True)
    return rec


def to_dev(x, dtype):
    return x.to("cuda", dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)


def param_dict_requires_grad(P):
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    return P
