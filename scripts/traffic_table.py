"""Per-kernel HBM traffic (PMC) against algorithmic bytes for the top kernels of a bench line.

  python scripts/traffic_table.py <bench.json> [profiles/pmc_traffic.json] [top]

Algorithmic bytes per launch = the bench's live HIP-event figure (roofline.kernels[k].gbs x avg_us); PMC bytes per
launch from scripts/pmc_traffic.py (FETCH_SIZE x 2 KiB + WRITE_SIZE x 1 KiB, gfx950 corrections). ratio > 1 means
bytes the design re-reads or spills; < 1 means L2 / Infinity-Cache reuse (memory-side counters do not see L2 hits
but include MALL hits)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (name matching between bench labels and rocprof symbols)

doc = json.loads(Path(sys.argv[1]).read_text())
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ks = doc["roofline"]["kernels"]
rows = sorted(ks.items(), key=lambda kv: -kv[1]["ms_total"])[:top]
print("| kernel | launches (timed) | avg us | algorithmic MB / launch | PMC MB / launch | PMC / algorithmic |")
print("|---|---|---|---|---|---|")
for name, k in rows:
    alg = k["gbs"] * 1e9 * k["avg_us"] * 1e-6 if k.get("gbs") else None
    pmc, _ = bench.pmc_traffic(name)
    ratio = f"{pmc / alg:.2f}" if pmc and alg else "—"
    print(f"| `{name[:70]}` | {k['launches']} | {k['avg_us']:.1f} | {alg / 1e6:.1f} | "
          f"{'—' if pmc is None else f'{pmc / 1e6:.1f}'} | {ratio} |" if alg else
          f"| `{name[:70]}` | {k['launches']} | {k['avg_us']:.1f} | — | {'—' if pmc is None else f'{pmc / 1e6:.1f}'} | — |")
