"""torch.cat(dim=1) on NHWC bf16 (reference Concat, nn/modules/conv.py:322-335): the pieces not written in place by
their producers are copied in one adr_copy_pieces launch; bitwise torch.cat, forward and the zero-copy backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chans", [(64, 64), (32, 128, 16), (8, 8, 8, 8, 8, 8, 8, 8, 8)])
def test_cat_pieces_bitwise(chans):
    from adrefine import kernels as K
    torch.manual_seed(0)
    xs = [torch.randn(3, c, 13, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
          .requires_grad_(True) for c in chans]
    y = K.cat(xs)
    ref = torch.cat([x.detach() for x in xs], 1)
    assert torch.equal(y, ref)
    g = torch.randn_like(ref)
    y.backward(g)
    off = 0
    for x, c in zip(xs, chans):
        assert torch.equal(x.grad, g[:, off:off + c])
        off += c
