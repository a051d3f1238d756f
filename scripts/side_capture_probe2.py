"""Probe: fork/join onto a second stream from inside an autograd backward (the engine's device thread) under
hipGraph capture, in the default ('global') and 'relaxed' capture modes. usage: python scripts/side_capture_probe2.py"""
import faulthandler
import sys

faulthandler.enable()
import torch

dev = torch.device("cuda", 0)
side = torch.cuda.Stream(dev)
keep = []


class F(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x * 2

    @staticmethod
    def backward(ctx, g):
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        keep.append(g)
        with torch.cuda.stream(side):
            t = g * 3  # allocation + kernel on the side stream
            keep.append(t)
        return g * 2


def body(x):
    y = F.apply(x).sum()
    y.backward()
    torch.cuda.current_stream().wait_stream(side)
    keep.clear()


x = torch.randn(1 << 16, device=dev, requires_grad=True)
body(x)
torch.cuda.synchronize()
mode = sys.argv[1] if len(sys.argv) > 1 else "global"
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode=mode):
    body(x)
g.replay()
torch.cuda.synchronize()
print("backward-thread fork/join capture ok:", mode, flush=True)
