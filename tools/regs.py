"""Per-kernel VGPRs / spills / occupancy of a libhipgp translation unit (hipcc
-Rpass-analysis=kernel-resource-usage).  Usage: python tools/regs.py hgp_pass_f32.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize",
       "-DHGP_CMAX_STRIDED=8", "-DHGP_MINW_STRIDED=2", "-DHGP_MINW_ROW=2", "-c", src, "-o", "/tmp/_regs.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="hipgp_amd/csrc").stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+):\s*(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if filt in k:
        print(f"{k[:70]:70s} vgpr {v.get('VGPRs', '?'):>4} spill {v.get('VGPRs Spill', '?'):>4} "
              f"occ {v.get('Occupancy [waves/SIMD]', '?')}")
