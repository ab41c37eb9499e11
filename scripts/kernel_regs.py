"""Per-kernel register / occupancy report from a hipcc ``-save-temps`` device .s
(the compiler's own ``; NumVgprs`` / ``; Occupancy`` remarks), to check a code
change does not push a kernel over an occupancy step.

    hipcc ... -c csrc/X.hip -save-temps=obj -o /tmp/X.o
    python scripts/kernel_regs.py /tmp/X-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import subprocess
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^; Occupancy: (\d+)", s, re.M | re.S):
    name, body, occ = m.group(1), m.group(2), m.group(3)
    v = re.search(r"; NumVgprs: (\d+)", body)
    sp = re.search(r"; ScratchSize: (\d+)", body)
    lds = re.search(r"; LDSByteSize: (\d+)", body)
    try:
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except Exception:
        dn = name
    if flt in dn:
        print(f"vgpr={v.group(1) if v else '?':>4s} occ={occ} scratch={sp.group(1) if sp else '?'} "
              f"lds={lds.group(1) if lds else '?'}  {dn[:110]}")
