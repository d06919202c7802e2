"""Per-kernel register / spill / occupancy table for route.hip (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "ddr_amd/csrc/route.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-x", "hip", "-c", src, "-o", "/tmp/_regs.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    s = m.group(1)
    if s.startswith("Function Name:"):
        cur = {"name": s.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in s:
        k, v = s.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if "route_" not in r["name"] and "gather" not in r["name"]:
        continue
    n = r["name"].replace("_ZN3ddr", "").replace("EEEvNS_9RouteArgsE", "")
    print(f'{n:42s} VGPR {r.get("VGPRs","?"):>4} spillV {r.get("VGPRs Spill","?"):>4} '
          f'SGPR {r.get("TotalSGPRs","?"):>4} spillS {r.get("SGPRs Spill","?"):>4} '
          f'scratch {r.get("ScratchSize [bytes/lane]","?"):>4} occ {r.get("Occupancy [waves/SIMD]","?")}')
