"""Per-step view of a rocprofv3 kernel-trace CSV (steps delimited by the optimizer kernel),
and a per-kernel diff of two steps (e.g. an eager step against a HIP-graph replay).

    python scripts/trace_steps.py TRACE.csv                 # every step: kernels, wall, busy, gaps
    python scripts/trace_steps.py TRACE.csv --diff I J      # step J minus step I, per kernel name
"""
import argparse
import collections
import csv
import re


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\((?!\().*$", "", n)
    return re.sub(r"^void ", "", n)[:100]


def steps(rows, marker):
    idx = [i for i, r in enumerate(rows) if re.search(marker, r[2])]
    return [rows[a + 1:b + 1] for a, b in zip(idx[:-1], idx[1:])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default=r"(adam|sgd)_kernel")
    ap.add_argument("--diff", nargs=2, type=int, default=None)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    st = steps(load(a.csv), a.marker)
    if a.diff is None:
        for i, sel in enumerate(st):
            wall = (sel[-1][1] - sel[0][0]) / 1e6
            busy = sum(e - s for s, e, _ in sel) / 1e6
            gaps = [sel[k + 1][0] - sel[k][1] for k in range(len(sel) - 1)]
            print(f"step {i:3d}: kernels={len(sel):5d} wall_ms={wall:8.2f} busy_ms={busy:8.2f} "
                  f"idle_ms={sum(g for g in gaps if g > 0) / 1e6:7.2f}")
        return

    def per_kernel(sel):
        c, t = collections.Counter(), collections.defaultdict(float)
        for s, e, n in sel:
            k = short(n)
            c[k] += 1
            t[k] += (e - s) / 1e6
        return c, t

    (ca, ta), (cb, tb) = per_kernel(st[a.diff[0]]), per_kernel(st[a.diff[1]])
    print(f"step {a.diff[1]} - step {a.diff[0]}: busy {sum(tb.values()) - sum(ta.values()):+.3f} ms, "
          f"kernels {sum(cb.values()) - sum(ca.values()):+d}")
    for k in sorted(set(ca) | set(cb), key=lambda k: -abs(tb[k] - ta[k]))[:a.top]:
        print(f"{cb[k] - ca[k]:+4d} calls {tb[k] - ta[k]:+7.3f} ms  ({ta[k]:7.3f} -> {tb[k]:7.3f})  {k}")


if __name__ == "__main__":
    main()
