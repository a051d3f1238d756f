"""Dev A/B helper: run a module fixture through adrefine (bf16 by default) and print relative-L2 errors of
outputs, input grads and the worst parameter-grad norms vs the golden fixture. Select the library with
ADR_LIB / ADR_HEADER to compare two builds."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "yolo-ad-refine_amd", ROOT / "tests", ROOT / "oracle", ROOT):
    sys.path.insert(0, str(p))
from conftest import golden  # noqa: E402
from gpu_util import load_recipe_into, to_dev  # noqa: E402
from recipe import seeded_randn  # noqa: E402
from test_gpu_blocks import SEEDS  # noqa: E402


def main(name, dtype=torch.bfloat16):
    from adrefine.nn.modules.head import AYHead
    from adrefine.nn.modules import block as B
    mods = {"ayhead": lambda: AYHead(80, [128, 128, 128]), "c2ptssa": lambda: B.C2PTSSA(256, 256, 1),
            "c3k2_mlca": lambda: B.C3k2_MLCA(128, 128, 1, False)}
    m = mods[name]()
    if name == "ayhead":
        m.stride = torch.tensor([8.0, 16.0, 32.0])
    g = golden(f"mod_{name}")
    load_recipe_into(m)
    m = m.cuda().train()
    ins, i = [], 0
    while f"in{i}_shape" in g:
        ins.append(to_dev(seeded_randn(*[int(v) for v in g[f"in{i}_shape"]], seed=int(g[f"in{i}_seed"])), dtype))
        i += 1
    out = m(ins) if name == "ayhead" else m(ins[0])
    outs = out if isinstance(out, (list, tuple)) else [out]
    gen = torch.Generator().manual_seed(SEEDS[name] + 1)
    gouts = [torch.randn(o.shape, generator=gen) for o in outs]
    torch.autograd.backward(list(outs), [gg.to("cuda", dtype).contiguous(memory_format=torch.channels_last)
                                         for gg in gouts])
    rl = lambda a, b: float((a.float().cpu().double() - torch.as_tensor(b).double()).norm() / torch.as_tensor(b).double().norm())  # noqa
    for j, o in enumerate(outs):
        print(f"out{j} relL2 {rl(o, g[f'out{j}']):.4e}")
    for j, x in enumerate(ins):
        print(f"gin{j} relL2 {rl(x.grad, g[f'gin{j}']):.4e}")
    ref = dict(zip([str(k) for k in g["param_grad_norms_keys"]], g["param_grad_norms"]))
    params = dict(m.named_parameters())
    errs = sorted(((abs(float(params[k].grad.norm()) - v) / (v + 1e-12), k) for k, v in ref.items()
                   if params[k].grad is not None), reverse=True)
    for e, k in errs[:6]:
        print(f"param {k} norm rel err {e:.3e}")


if __name__ == "__main__":
    main(sys.argv[1])
