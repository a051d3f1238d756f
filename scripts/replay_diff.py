"""Per-kernel difference of two replay_breakdown.py tables (A - B), largest changes first.
usage: python scripts/replay_diff.py A_replay.md B_replay.md [n]"""
import sys


def load(p):
    d = {}
    for ln in open(p):
        parts = [x.strip() for x in ln.strip().strip("|").split("|")]
        if len(parts) == 4:
            try:
                d[parts[0]] = (float(parts[1]), int(parts[2]))
            except ValueError:
                pass
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 15
rows = sorted((a.get(k, (0, 0))[0] - b.get(k, (0, 0))[0], k) for k in set(a) | set(b))
for dt, k in rows[:n] + [(None, "...")] + rows[-n:]:
    if dt is None:
        print("...")
        continue
    ta, na = a.get(k, (0, 0))
    tb, nb = b.get(k, (0, 0))
    print(f"{dt:+.3f}  A {ta:.3f}/{na}  B {tb:.3f}/{nb}  {k[:110]}")
