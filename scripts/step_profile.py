"""Per-step kernel breakdown from a rocprofv3 kernel-trace CSV: a full training step is
delimited by the optimizer kernel (adam_kernel / sgd_kernel); --window picks which one.

Usage: python scripts/step_profile.py <run_kernel_trace.csv> [--top 30]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--marker", default=r"(adam|sgd)_kernel")
ap.add_argument("--window", type=int, default=2,
                help="the step ending at the optimizer dispatch this many places from the end (bench.py's "
                     "last window also holds the after-timing checksums)")
a = ap.parse_args()

rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
idx = [i for i, r in enumerate(rows) if re.search(a.marker, r[2])]
if len(idx) < 2:
    raise SystemExit("need >= 2 optimizer steps in the trace")
w = min(a.window, len(idx) - 1)
sel = rows[idx[-w - 1] + 1: idx[-w] + 1]


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\((?!\().*$", "", n) if not n.startswith("void") else n
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:100]


tot = collections.defaultdict(float)
cnt = collections.Counter()
for s, e, n in sel:
    k = short(n)
    tot[k] += (e - s) / 1e6
    cnt[k] += 1
wall = (sel[-1][1] - sel[0][0]) / 1e6
busy = sum(tot.values())
print(f"one step: kernels={len(sel)} wall_ms={wall:.2f} busy_ms={busy:.2f}")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[: a.top]:
    print(f"{v:9.3f} ms {100 * v / busy:5.1f}% {cnt[k]:5d}  {k}")
