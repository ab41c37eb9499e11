"""Summarise a rocprofv3 kernel-trace CSV over the last N training steps.

Usage: python scripts/trace_summary.py <kernel_trace.csv> [--steps N] [--marker SUBSTR]
Steps are delimited by occurrences of a marker kernel (default: the last
kernel name of the optimizer step, auto-detected as the most frequent
kernel whose count == number of steps) -- simpler: we split on gaps.
"""
import csv, sys, collections, argparse

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--marker", default=None, help="substring of a kernel launched once per step (first kernel of a step)")
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()

rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
if a.marker:
    idx = [i for i, r in enumerate(rows) if a.marker in r[2]]
    start = idx[-a.steps - 1] if len(idx) > a.steps else 0
    end = idx[-1]
    sel = rows[start:end]
else:
    # use the last fraction of the trace
    n = len(rows)
    sel = rows[int(n * (1 - 0.2)):]
tot = collections.Counter(); cnt = collections.Counter()
for s, e, name in sel:
    short = name[:110]
    tot[short] += e - s; cnt[short] += 1
wall = sel[-1][1] - sel[0][0]
busy = sum(tot.values())
print(f"kernels={len(sel)} wall_ms={wall/1e6:.2f} busy_ms={busy/1e6:.2f} per_step_wall_ms={wall/1e6/max(a.steps,1):.2f}")
for k, v in tot.most_common(a.top):
    print(f"{v/1e6:9.3f} ms {cnt[k]:5d}  {k}")
