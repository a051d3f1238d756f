"""Probe: many forks onto one side stream (one per backward node, as the WGRAD side stream does) and one join,
under hipGraph capture. usage: python scripts/side_capture_probe3.py <nodes> [alloc|noalloc] [joineach]"""
import faulthandler
import sys

faulthandler.enable()
import torch

dev = torch.device("cuda", 0)
side = torch.cuda.Stream(dev)
keep = []
nodes = int(sys.argv[1])
alloc = sys.argv[2] == "alloc"
joineach = len(sys.argv) > 3
acc = torch.zeros(1 << 16, device=dev)


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
            if alloc:
                t = g * 3
                keep.append(t)
            else:
                acc.add_(g)
        if joineach:
            main.wait_stream(side)
        return g * 2


def body(x):
    y = x
    for _ in range(nodes):
        y = F.apply(y)
    y.sum().backward()
    torch.cuda.current_stream().wait_stream(side)
    keep.clear()


x = torch.randn(1 << 16, device=dev, requires_grad=True)
body(x)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body(x)
g.replay()
torch.cuda.synchronize()
print("ok", sys.argv[1:], flush=True)
