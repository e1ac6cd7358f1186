"""Static check of libhipgp's gfx950 code for the VMEM store-data hazard behind the fp64
contiguous-line race (profiles/r3_buf64_race.txt).

A buffer store of more than 8 bytes (dwordx3 / dwordx4) reads its data VGPRs after issue;
a VALU instruction in the next cycle that overwrites them can change the stored data of the
last lanes.  LLVM's hazard recognizer inserts the wait state only when the store's soffset
is not an SGPR (GCNHazardRecognizer::createsVALUHazard), so a 128-bit raw-buffer store with an
SGPR soffset followed directly by a VALU write of its data is emitted unprotected.

Usage: python tools/hazard_lint.py [lib.so]   -> prints each hit, exit 1 if any.
Also used by tests/test_hazard_lint_cpu.py.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
STORE = re.compile(r"^\s*buffer_store_dword(x3|x4)\s+v\[(\d+):(\d+)\],\s*\S+,\s*s\[\d+:\d+\],\s*(\S+)")
VALU = re.compile(r"^\s*v_\w+\s+(v\[(\d+):(\d+)\]|v(\d+))")


def code_objects(lib, tmp):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin."""
    fat = os.path.join(tmp, "fat.bin")
    # objcopy writes its output file even when only dumping: give it a scratch one (with the
    # input alone it rewrites the library in place -- under a process that has it mapped)
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "scratch.so")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = []
    i = data.find(MAGIC)
    while i != -1:
        starts.append(i)
        i = data.find(MAGIC, i + 1)
    starts.append(len(data))
    out = []
    for k in range(len(starts) - 1):
        b = os.path.join(tmp, f"b{k}.bin")
        co = os.path.join(tmp, f"b{k}.co")
        open(b, "wb").write(data[starts[k]:starts[k + 1]])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={b}",
                            f"--output={co}", "--unbundle"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def scan(asm_lines):
    """Hits: (store line, next instruction) where a >8-byte buffer store with an SGPR soffset
    is directly followed by a VALU write of one of its data VGPRs."""
    hits = []
    insts = [ln for ln in asm_lines if ln.strip() and not ln.lstrip().startswith(("//", ";")) and not ln.rstrip().endswith(":")]
    for j, ln in enumerate(insts[:-1]):
        m = STORE.match(ln)
        if not m or not m.group(4).startswith("s"):
            continue
        lo, hi = int(m.group(2)), int(m.group(3))
        nxt = insts[j + 1]
        v = VALU.match(nxt)
        if not v:
            continue
        if v.group(2) is not None:
            dlo, dhi = int(v.group(2)), int(v.group(3))
        else:
            dlo = dhi = int(v.group(4))
        if dlo <= hi and dhi >= lo:
            hits.append((ln.split("//")[0].strip(), nxt.split("//")[0].strip()))
    return hits


def lint(lib):
    with tempfile.TemporaryDirectory() as tmp:
        hits, nstores = [], 0
        for co in code_objects(lib, tmp):
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout.splitlines()
            nstores += sum(1 for ln in dis if "buffer_store_dwordx" in ln)
            hits += scan(dis)
        return hits, nstores


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "hipgp_amd", "libhipgp.so")
    hits, n = lint(lib)
    for s, v in hits:
        print(f"HAZARD: {s}  ->  {v}")
    print(f"{os.path.basename(lib)}: {n} buffer stores scanned, {len(hits)} unprotected >8-byte store-data hazards")
    sys.exit(1 if hits else 0)
