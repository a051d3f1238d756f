"""bf16 parameter-gradient bisection: run the net701_grads_320 backward in bf16 once per environment toggle
(each in its own child process, since the toggles are read at import) and print the relative L2 error of every
fixture gradient against the fp32 reference.   python scripts/grad_bisect.py [ENV=V ...]"""
import json
import os
import subprocess
import sys

TOGGLES = ["", "ADR_BN_XF_BWD=0", "ADR_DEFER_DOT=0", "ADR_DEFER_COLSUM=0", "ADR_DEFER_ADD=0", "ADR_FANOUT_SINK=0",
           "ADR_SEED_CAT=0", "ADR_DCN_FUSED=0", "ADR_GN_FUSED=0", "ADR_DEFER_GN=0", "ADR_EVAL_FUSE=0"]

CHILD = r"""
import sys, json
sys.path.insert(0, "tests"); sys.path.insert(0, "yolo-ad-refine_amd"); sys.path.insert(0, "oracle")
import torch
from conftest import golden
import test_gpu_grads as T
g = golden("net701_grads_320")
ref = T._ref(g)
_, mine = T._hip_grads(torch.bfloat16, g)
rel = {k: float((mine[k] - r).norm() / (r.norm() + 1e-30)) for k, r in ref.items()}
print("JSON" + json.dumps(rel))
"""


def main():
    toggles = sys.argv[1:] or TOGGLES
    rows = {}
    for t in toggles:
        env = dict(os.environ)
        for kv in filter(None, t.split(",")):
            k, v = kv.split("=")
            env[k] = v
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in p.stdout.splitlines() if x.startswith("JSON")]
        if p.returncode or not line:
            print(t or "default", "FAILED", p.returncode, p.stderr[-2000:], flush=True)
            break
        rows[t or "default"] = json.loads(line[0][4:])
        r = rows[t or "default"]
        worst = sorted(r.items(), key=lambda kv: -kv[1])[:6]
        print(t or "default", json.dumps({k: round(v, 4) for k, v in worst}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/grad_bisect.json", "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
