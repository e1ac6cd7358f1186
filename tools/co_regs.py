"""VGPRs / AGPRs / spills / LDS of the kernels in a built libhipgp object, from the gfx950 code
object's metadata notes (no recompilation).  Usage:
    python tools/co_regs.py [hipgp_amd/csrc/build/hgp_pass_f32.o] [name filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj = sys.argv[1] if len(sys.argv) > 1 else "hipgp_amd/csrc/build/hgp_pass_f32.o"
filt = sys.argv[2] if len(sys.argv) > 2 else ""
with tempfile.TemporaryDirectory() as td:
    tmp = os.path.join(td, os.path.basename(obj))
    with open(obj, "rb") as a, open(tmp, "wb") as b:
        b.write(a.read())
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tmp], capture_output=True, check=True, cwd=td)
    co = [f for f in os.listdir(td) if "gfx950" in f][0]
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(td, co)], capture_output=True,
                           text=True, check=True).stdout
    names = subprocess.run(["c++filt"], input="\n".join(re.findall(r"\.name:\s+(\S+)", notes)),
                           capture_output=True, text=True).stdout.splitlines()
keys = ("vgpr_count", "agpr_count", "vgpr_spill_count", "group_segment_fixed_size", "private_segment_fixed_size")
cur, rows = {}, []
for line in notes.splitlines():
    m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "name":
        cur["name"] = v
    elif k in keys:
        cur[k] = v
    if k == "wavefront_size" and "name" in cur:
        rows.append(cur)
        cur = {}
    elif "name" in cur and all(kk in cur for kk in keys):
        rows.append(cur)
        cur = {}
dem = dict(zip(re.findall(r"\.name:\s+(\S+)", notes), names))
for r in rows:
    n = dem.get(r["name"], r["name"])
    if filt in n:
        print(f"{n[:72]:72s} vgpr {r.get('vgpr_count', '?'):>4} agpr {r.get('agpr_count', '?'):>3} "
              f"spill {r.get('vgpr_spill_count', '?'):>3} lds {r.get('group_segment_fixed_size', '?'):>6} "
              f"scratch {r.get('private_segment_fixed_size', '?')}")
