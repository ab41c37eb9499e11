"""Append the bench.py JSON records found in gpurun_out logs to profiles/bench_runs_round6.jsonl,
tagged with the log name (the gpurun call tag) and a note.

    python scripts/keep_bench.py NOTE gpurun_out/r5a_bench_*.txt ...
"""
import json
import sys
from pathlib import Path

OUT = Path(__file__).resolve().parents[1] / "profiles" / "bench_runs_round6.jsonl"


def main():
    note, files = sys.argv[1], sys.argv[2:]
    n = 0
    with OUT.open("a") as fo:
        for f in files:
            for line in Path(f).read_text().splitlines():
                if line.startswith("{") and '"metric"' in line:
                    rec = json.loads(line)
                    rec["run"] = Path(f).stem
                    rec["note"] = note
                    fo.write(json.dumps(rec) + "\n")
                    n += 1
    print(f"kept {n} record(s) in {OUT}")


if __name__ == "__main__":
    main()
