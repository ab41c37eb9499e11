"""Per-kernel-family hardware-counter table for ONE training step from the
rocprofv3 --pmc passes written by scripts/pmc_passes.sh.

The step is delimited by the optimizer kernel (sgd_kernel / adam_kernel): the
last complete step between two optimizer dispatches of each pass.

    python scripts/pmc_summary.py gpurun_out/TAG_pmc1 gpurun_out/TAG_pmc2 ... [--top 25]

Columns (sums over the step's dispatches of a family):
  ms      kernel time in the profiled pass (End - Start per dispatch; profiled runs
          serialise dispatches and run at a slightly different clock)
  GHz     GRBM_GUI_ACTIVE / 8 XCDs / time (calibrated: a 265 us GEMM reads 2.36-2.41)
  MFMA%   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
  TF/s    (SQ_INSTS_VALU_MFMA_MOPS_BF16 + _F8) * 512 FLOP / time (calibrated: 12.85 M
          16x16x32 bf16 MFMAs = 411 M MOPS = 210 GFLOP)
  ldsconf SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (conflict cycles per LDS instruction)
  L2hit   TCC_HIT / (TCC_HIT + TCC_MISS)
  fetchMB FETCH_SIZE (KiB) / 1024  -- NB gfx950 FETCH_SIZE reads ~1/2 of wide streams (guide §7)
  writeMB WRITE_SIZE (KiB) / 1024
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def short(n: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([\w:]+(?:<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:90]


def load_pass(d: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return {}
    rows = list(csv.DictReader(open(files[0])))
    if not rows:
        return {}
    kcol = next(c for c in rows[0] if c.lower() in ("kernel_name", "kernel-name"))
    dcol = next(c for c in rows[0] if c.lower() in ("dispatch_id", "correlation_id"))
    ncol = next(c for c in rows[0] if c.lower() == "counter_name")
    vcol = next(c for c in rows[0] if c.lower() == "counter_value")
    per = collections.defaultdict(dict)  # dispatch -> {counter: value}
    names = {}
    for r in rows:
        did = int(r[dcol])
        names[did] = r[kcol]
        per[did][r[ncol]] = per[did].get(r[ncol], 0.0) + float(r[vcol])
        if "Start_Timestamp" in r:
            per[did]["_ns"] = float(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    order = sorted(per)
    opt = [d for d in order if re.search(r"(sgd|adam)_kernel", names[d])]
    # the window ending at the optimizer dispatch WINDOW places from the end: bench.py's last
    # window holds its after-timing work (the rank-consistency checksums), so 2 by default
    w = int(os.environ.get("PMC_WINDOW", "2"))
    if len(opt) >= w + 1:
        order = [d for d in order if opt[-w - 1] < d <= opt[-w]]
    elif len(opt) >= 2:
        order = [d for d in order if opt[-2] < d <= opt[-1]]
    out = collections.defaultdict(lambda: collections.Counter())
    cnt = collections.Counter()
    for d in order:
        k = short(names[d])
        cnt[k] += 1
        for c, v in per[d].items():
            out[k][c] += v
        out[k]["_n"] += 1
    return out, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--rate", default="", help="comma-separated SQ counters printed as %% of SIMD-cycles "
                                                 "(counter / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), e.g. "
                                                 "SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS")
    a = ap.parse_args()
    rates = [r for r in a.rate.split(",") if r]
    fam = collections.defaultdict(collections.Counter)
    calls = collections.Counter()
    for d in a.dirs:
        r = load_pass(d)
        if not r:
            continue
        out, cnt = r
        for k, c in out.items():
            c = collections.Counter(c)
            if "_ns" in fam[k]:  # keep the first pass's time only
                del c["_ns"]
            fam[k].update(c)
            calls[k] = max(calls[k], cnt[k])
    key = "SQ_BUSY_CYCLES" if any("SQ_BUSY_CYCLES" in c for c in fam.values()) else "SQ_WAVE_CYCLES"
    ranked = sorted(fam, key=lambda k: -fam[k].get("_ns", fam[k].get("GRBM_GUI_ACTIVE", 0)))
    nan = float("nan")
    tot_ns = sum(c.get("_ns", 0) for c in fam.values())
    print(f"step kernel time in the profiled pass: {tot_ns / 1e6:.2f} ms over {sum(calls.values())} dispatches")
    hdr = (f"{'kernel family':72s} {'calls':>5s} {'ms':>7s} {'GHz':>5s} {'MFMA%':>6s} {'TF/s':>6s} {'ldsconf':>7s} "
           f"{'L2hit':>6s} {'fetchMB':>8s} {'writeMB':>8s}" + "".join(f" {r[-12:]:>12s}" for r in rates))
    print(hdr)
    for k in ranked[: a.top]:
        c = fam[k]
        ns = c.get("_ns", 0)
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        ghz = cyc / ns if ns else nan
        mf = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc) if cyc else nan
        tf = (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0)) * 512 / ns / 1e3 \
            if ns else nan
        li = c.get("SQ_INSTS_LDS", 0)
        lc = c.get("SQ_LDS_BANK_CONFLICT", 0) / li if li else nan
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        hr = h / (h + m) if h + m else nan
        print(f"{k[:72]:72s} {calls[k]:5d} {ns / 1e6:7.3f} {ghz:5.2f} {mf:6.1f} {tf:6.0f} {lc:7.3f} {hr:6.3f} "
              f"{c.get('FETCH_SIZE', 0) / 1024:8.1f} {c.get('WRITE_SIZE', 0) / 1024:8.1f}" +
              "".join(f" {100 * c.get(r, 0) / (1024 * cyc) if cyc else nan:12.1f}" for r in rates))
    print("counters seen:", sorted({n for c in fam.values() for n in c}))


if __name__ == "__main__":
    main()
