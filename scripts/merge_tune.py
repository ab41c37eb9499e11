"""Merge fresh autotune entries (gpurun_out/tune_*.json, from `gpu_job.sh retune:NAME:ARGS`)
into the shipped table pytorch_distributed_template_amd/_lib/autotune_gfx950.json."""
import json
import sys
from pathlib import Path

SHIPPED = Path(__file__).resolve().parents[1] / "pytorch_distributed_template_amd" / "_lib" / "autotune_gfx950.json"


def main():
    table = json.loads(SHIPPED.read_text())
    changed = 0
    for f in sys.argv[1:]:
        new = json.loads(Path(f).read_text())
        for k, v in new.items():
            if table.get(k) != v:
                changed += 1
                print(f"{k}: {table.get(k)} -> {v}")
            table[k] = v
    SHIPPED.write_text(json.dumps(table, indent=0, sort_keys=True) + "\n")
    print(f"{changed} entries changed, {len(table)} total")


if __name__ == "__main__":
    main()
