"""Per-step GPU time by kernel family from a rocprofv3 --stats kernel_stats.csv of a bench.py run.
The number of profiled steps is taken from a once-per-step kernel (the det-loss classification-gradient kernel),
so warmup, capture and replay steps are all counted.  usage: python scripts/kernel_breakdown.py <kernel_stats.csv>"""
import csv
import sys
from collections import defaultdict

FAMILIES = [  # (family, substrings) — first match wins
    ("conv fwd/dgrad (adr_conv, MFMA)", ["conv_bf16_kernel", "conv3_kernel", "conv1_kernel", "conv_bf16_xf", "conv3_xf",
                                         "conv3w_kernel", "conv_bf16_act", "conv1_xf", "conv1_act", "conv3_act",
                                         "conv_fp8", "gemm_kernel", "stem_fwd", "conv_bf16_bst", "conv1_bst",
                                         "conv3_bst", "conv3w_bst", "dg2_kernel"]),
    ("conv wgrad (MFMA) + split-K reduce", ["wgrad_bf16_kernel", "wgrad_bf16_batched", "wgrad3_kernel", "wgrad3t_kernel",
                                            "wgrad_reduce", "stem_wgrad"]),
    ("BN/GN stats, finalize, affine+act", ["nc_reduce", "affine_act", "bn_finalize", "bn_bwd_finalize", "gn_",
                                           "partial_sum", "nc_collapse", "dot_reduce"]),
    ("elementwise / broadcast", ["ew_kernel", "bcast_", "axpy", "cast_kernel", "scale_"]),
    ("DCNv2 (im2col / col2im)", ["dcn_"]),
    ("attention / TSSA / EDFFN / ADyT / dwconv", ["attn_", "tssa", "edffn", "adyt", "dw_", "dyt", "ln_mix"]),
    ("pool / gate / MLCA / upsample", ["pool", "gate", "mlca", "axis_mean", "bilinear", "adapool", "mul_pixel",
                                       "group_mean", "fusion"]),
    ("loss (TAL + box/DFL/cls)", ["loss_", "tal_", "dfl", "det_"]),
    ("optimizer + weight packing", ["sgd_ema", "grad_sqnorm", "pack_weight", "opt_"]),
    ("PyTorch-native (autograd adds, fills)", ["at::native", "at::"]),
    ("HIP runtime copies / fills", ["__amd_rocclr"]),
]


def main(path):
    rows = list(csv.DictReader(open(path)))
    steps = next((int(r["Calls"]) for r in rows if "loss_cls_grad_kernel" in r["Name"]), None)
    if not steps:
        raise SystemExit("no once-per-step marker kernel in the profile")
    fam = defaultdict(lambda: [0.0, 0])
    for r in rows:
        name = r["Name"]
        f = next((f for f, keys in FAMILIES if any(k in name for k in keys)), "other")
        fam[f][0] += float(r["TotalDurationNs"]) / steps / 1e6
        fam[f][1] += int(r["Calls"]) / steps
    total = sum(v[0] for v in fam.values())
    print(f"{steps} profiled steps; GPU kernel time per step {total:.2f} ms")
    print("| family | ms / step | launches / step | share |\n|---|---|---|---|")
    for f, (ms, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"| {f} | {ms:.2f} | {n:.0f} | {100 * ms / total:.1f} % |")


if __name__ == "__main__":
    main(sys.argv[1])
