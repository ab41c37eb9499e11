"""Which kernels ran: one line per kernel name of a rocprofv3 kernel-trace CSV (count,
total ms), with library kernels flagged -- MIOpen (`miopen`, `MIOpen`, `naive_conv`,
`igemm`), rocBLAS/hipBLASLt (`Cijk_`) and PyTorch's own (`at::native`).

    python scripts/kernel_census.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import collections
import csv
import sys

LIB = (("miopen", "MIOpen"), ("MIOpen", "MIOpen"), ("naive_conv", "MIOpen"), ("igemm", "MIOpen"),
       ("Cijk_", "rocBLAS/hipBLASLt"), ("at::native", "torch"))


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    cnt, ms = collections.Counter(), collections.Counter()
    for r in rows:
        n = r["Kernel_Name"]
        cnt[n] += 1
        ms[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    flagged = collections.Counter()
    for n, c in sorted(cnt.items(), key=lambda kv: -ms[kv[0]]):
        tag = next((lib for pat, lib in LIB if pat in n), "")
        if tag:
            flagged[tag] += c
        print(f"{c:7d} {ms[n]:10.3f} ms  {tag:18s} {n[:110]}")
    print(f"total dispatches {sum(cnt.values())}; library kernels: {dict(flagged) or 'none'}")


if __name__ == "__main__":
    main()
