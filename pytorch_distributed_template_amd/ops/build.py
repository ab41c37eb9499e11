"""Build the HIP kernel library for gfx950 (in-tree, no JIT cache).

``python -m pytorch_distributed_template_amd.ops.build`` compiles every
``csrc/*.hip`` with ``hipcc --offload-arch=gfx950 -O3`` into objects under
``build/hip`` and links ``pytorch_distributed_template_amd/_lib/libpdt_hip.so``.
The library exposes a C ABI only (see ``csrc/pdt_common.h``) and is loaded
with ctypes by ``ops/native_ops.py`` -- no torch headers, no hipify.
Incremental: an object is rebuilt only when its source or a header changed.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]
ROOT = PKG.parent
CSRC = ROOT / "csrc"
OUT_DIR = PKG / "_lib"
LIB = OUT_DIR / "libpdt_hip.so"
OBJ_DIR = ROOT / "build" / "hip"
ARCH = os.environ.get("PDT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wno-unused-result"]


def _compile(src: Path, headers_mtime: float) -> Path:
    obj = OBJ_DIR / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, headers_mtime):
        return obj
    cmd = [HIPCC, *FLAGS, "-I", str(CSRC), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = True) -> Path:
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    sources = sorted(CSRC.glob("*.hip"))
    headers = list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc"))
    hm = max([h.stat().st_mtime for h in headers] + [0.0])
    with cf.ThreadPoolExecutor(max_workers=min(8, len(sources))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm), sources))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[pdt] built {LIB} from {len(sources)} sources", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
