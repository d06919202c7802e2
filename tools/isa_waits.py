"""List the vmcnt waits of a routing kernel's tick loop, by phase (DDR_PHASE_PROF markers).

    python tools/isa_waits.py [forward|backward] [KR] [extra -D flags ...]

Compiles route.hip for gfx950 (device only, -S) with -DDDR_PHASE_PROF=1 and prints, between
consecutive s_memtime markers, every s_waitcnt that includes vmcnt with the two preceding
instructions, so a wait that would drain the tick's prefetches stands out.
"""
import re
import subprocess
import sys
from pathlib import Path

kind = sys.argv[1] if len(sys.argv) > 1 else "forward"
kr = sys.argv[2] if len(sys.argv) > 2 else "4"
extra = sys.argv[3:]
src = Path(__file__).resolve().parents[1] / "ddr_amd" / "csrc"
out = Path("/tmp/isa_waits.s")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-unused-function", "-DDDR_PHASE_PROF=1", *extra, "-x", "hip",
       "--cuda-device-only", "-S", str(src / "route.hip"), "-o", str(out)]
subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
s = out.read_text()
name = re.findall(rf"^(_Z\w*route_{kind}_kernelIfLi{kr}\w*):", s, re.M)[0]
body = s[s.index(name + ":"):s.index(".Lfunc_end", s.index(name + ":"))].splitlines()
ins = [l.strip() for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
seg, counts = 0, {}
for i, l in enumerate(ins):
    if l.startswith("s_memtime"):
        seg += 1
        continue
    if l.startswith("s_waitcnt") and "vmcnt" in l:
        counts[seg] = counts.get(seg, 0) + 1
        print(f"seg {seg:3d}  {l:28s} <- {ins[i - 2][:50]} | {ins[i - 1][:50]}")
print("vmcnt waits per marker segment:", counts)
