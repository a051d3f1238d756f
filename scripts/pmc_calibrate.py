"""Calibrate the PMC byte counts (FETCH_SIZE / WRITE_SIZE) against kernels of this library whose HBM bytes are
known exactly, one per access pattern: 16-byte-per-lane NHWC streaming (adr_affine_act), 1-byte NCHW image reads
(adr_stem_conv_fwd_u8), fp32 -> bf16 conversion (adr_cast) and a bilinear GATHER (adr_dcn_fwd_bf16 with zero
offsets: every tap samples an integer neighbour, so its compulsory bytes are x + offsets/mask + w + y). Each kernel
cycles through buffer sets totalling > 512 MB, so no launch finds its inputs in the 256 MiB Infinity Cache.

  python scripts/pmc_calibrate.py run <out_dir>                                (under rocprofv3 --pmc, twice)
  python scripts/pmc_calibrate.py combine <fetch_dir> <write_dir> <known.json> <out.json>"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))


def run(out_dir):
    import ctypes

    import torch

    from adrefine import kernels as K
    from adrefine.native import lib
    dev = torch.device("cuda", 0)
    st = K.stream()
    known = {}
    sets = 4
    # 1. affine_act: bf16 NHWC 64 x 160^2 x 64 in, same out (16 B / lane loads and stores)
    N, HW, C = 64, 160 * 160, 64
    xs = [torch.randn(N * HW * C, device=dev).bfloat16() for _ in range(sets)]
    zs = [torch.empty_like(x) for x in xs]
    sc, sh = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    for r in range(12):
        i = r % sets
        lib.adr_affine_act(K.BF16, ctypes.c_void_p(xs[i].data_ptr()), C, 0, ctypes.c_void_p(zs[i].data_ptr()), C, 0,
                           K.fptr(sc), K.fptr(sh), 0, K.ACT["silu"], N, HW, C, st)
    known["affine_act_kernel"] = {"read": 2 * N * HW * C + 8 * C, "write": 2 * N * HW * C,
                                  "pattern": "16 B/lane NHWC streaming"}
    del xs, zs
    # 2. stem forward on the uint8 batch: 64 x 3 x 640^2 bytes in, 64 x 320^2 x 16 bf16 out
    N, H, W, Kc = 64, 640, 640, 16
    imgs = [torch.randint(0, 255, (N, 3, H, W), dtype=torch.uint8, device=dev) for _ in range(sets)]
    ys = [torch.empty(N * 320 * 320 * Kc, dtype=torch.bfloat16, device=dev) for _ in range(sets)]
    w = torch.randn(Kc * 27, device=dev) * 0.1
    for r in range(12):
        i = r % sets
        lib.adr_stem_conv_fwd_u8(ctypes.c_void_p(imgs[i].data_ptr()), N, H, W, K.fptr(w), Kc,
                                 ctypes.c_void_p(ys[i].data_ptr()), Kc, None, st)
    known["stem_fwd_kernel"] = {"read": N * 3 * H * W + 4 * Kc * 27, "write": 2 * N * 320 * 320 * Kc,
                                "pattern": "1 B NCHW image rows (3x3 s2 windows)"}
    del imgs, ys
    # 3. cast fp32 -> bf16, 64 Mi elements
    n = 64 << 20
    srcs = [torch.randn(n, device=dev) for _ in range(sets)]
    dsts = [torch.empty(n, dtype=torch.bfloat16, device=dev) for _ in range(sets)]
    for r in range(12):
        i = r % sets
        lib.adr_cast(K.F32, ctypes.c_void_p(srcs[i].data_ptr()), K.BF16, ctypes.c_void_p(dsts[i].data_ptr()), n, st)
    known["cast"] = {"read": 4 * n, "write": 2 * n, "pattern": "fp32 -> bf16 streaming"}
    del srcs, dsts
    # 4. DCNv2 forward gather, zero offsets, mask logits 0: 64 x 80^2 x 128 -> 128
    N, H, W, C = 64, 80, 80, 128
    xs = [torch.randn(N * H * W * C, device=dev).bfloat16() for _ in range(sets)]
    oms = [torch.zeros(N * H * W * 32, dtype=torch.bfloat16, device=dev) for _ in range(sets)]
    ys = [torch.empty(N * H * W * C, dtype=torch.bfloat16, device=dev) for _ in range(sets)]
    wk = (torch.randn(C * 9 * C, device=dev) * 0.02).bfloat16()
    for r in range(12):
        i = r % sets
        lib.adr_dcn_fwd_bf16(ctypes.c_void_p(xs[i].data_ptr()), C, ctypes.c_void_p(oms[i].data_ptr()), 32,
                             ctypes.c_void_p(wk.data_ptr()), ctypes.c_void_p(ys[i].data_ptr()), C, N, H, W, C, C, st)
    known["dcn_fwd"] = {"read": 2 * N * H * W * (C + 32) + 2 * 9 * C * C, "write": 2 * N * H * W * C,
                        "pattern": "bilinear gather (integer taps), 3x3 neighbourhood re-reads"}
    torch.cuda.synchronize()
    Path(out_dir).mkdir(parents=True, exist_ok=True)
    (Path(out_dir) / "known.json").write_text(json.dumps(known, indent=1))
    print("ok", list(known))


def combine(fdir, wdir, known_f, out):
    sys.path.insert(0, str(ROOT / "scripts"))
    from pmc_traffic import load
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    known = json.loads(Path(known_f).read_text())
    res = {}
    for key, kb in known.items():
        names = [n for n in fetch if key in n]
        if len(names) != 1:
            res[key] = {"error": f"{len(names)} matching kernels"}
            continue
        n = names[0]
        fv = list(fetch[n].values())
        wv = list(write.get(n, {}).values())
        f_kib = sum(fv) / len(fv)
        w_kib = sum(wv) / len(wv) if wv else None
        res[key] = {"kernel": n, "pattern": kb["pattern"], "launches": len(fv),
                    "alg_read": kb["read"], "alg_write": kb["write"],
                    "fetch_kib": round(f_kib), "write_kib": None if w_kib is None else round(w_kib),
                    "read_factor": round(kb["read"] / (1024 * f_kib), 3),  # alg read bytes per FETCH KiB / 1024
                    "write_factor": None if not w_kib else round(kb["write"] / (1024 * w_kib), 3)}
    doc = {"what": "bytes per FETCH_SIZE (resp. WRITE_SIZE) KiB x 1/1024, per access pattern: 2.0 means the "
                   "counter reports half of the bytes (the gfx950 wide-load case of MI355X_MICROARCH.md)",
           "kernels": res}
    Path(out).write_text(json.dumps(doc, indent=1))
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        combine(*sys.argv[2:6])
