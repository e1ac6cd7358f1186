"""Static instruction mix of libhipgp kernels from the built gfx950 code object (no GPU):
VALU split into packed / scalar fp arithmetic (the FFT's butterflies, twiddle products, spectrum
multiply) and integer / move / select work (index, LDS-address, twiddle-index math), plus LDS,
memory, scalar and branch instructions.  The FFT kernels are straight-line code (every loop over
stages / points unrolled), so the static counts track the per-wave dynamic ones that SQ_INSTS_*
counters give (tools/pmc_pass.sh).

    python tools/isa_mix.py [object] [kernel-name regex] [--list]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj, td):
    tmp = os.path.join(td, os.path.basename(obj))
    with open(obj, "rb") as a, open(tmp, "wb") as b:
        b.write(a.read())
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tmp], capture_output=True, check=True, cwd=td)
    return os.path.join(td, [f for f in os.listdir(td) if "gfx950" in f][0])


def classify(mn):
    if mn.startswith("v_pk_") and any(k in mn for k in ("_f32", "_f16")):
        return "valu_fp_packed"
    if mn.startswith("v_") and re.search(r"_(f32|f64)\b|_f32_|_f64_", mn) and not mn.startswith(("v_cvt", "v_cmp", "v_cndmask")):
        if any(k in mn for k in ("fma", "mul", "add", "sub", "mac", "max", "min")):
            return "valu_fp_scalar"
    if mn.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")):
        return "valu_move"
    if mn.startswith(("v_cndmask", "v_cmp")):
        return "valu_select_cmp"
    if mn.startswith("v_"):
        return "valu_int_addr_other"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_setprio")):
        return "sync_wait"
    if mn.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if mn.startswith("s_"):
        return "salu_smem"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    obj = args[0] if args else "hipgp_amd/csrc/build/hgp_pass_f32.o"
    pat = re.compile(args[1] if len(args) > 1 else ".")
    with tempfile.TemporaryDirectory() as td:
        co = code_object(obj, td)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                             text=True, check=True).stdout
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+([a-z_0-9]+)(\s|$)", line)
        if m:
            funcs[cur].append(m.group(1))
    names = list(funcs)
    dem = dict(zip(names, subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                                         text=True).stdout.splitlines()))
    for mangled, ins in funcs.items():
        name = dem.get(mangled, mangled)
        if not pat.search(name) or not ins:
            continue
        if "--list" in sys.argv:
            print(name)
            continue
        c = collections.Counter(classify(i) for i in ins)
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        print(f"{name}\n  total {len(ins)}  VALU {valu}: " +
              ", ".join(f"{k} {c[k]} ({100 * c[k] / max(valu, 1):.0f}%)" for k in sorted(c) if k.startswith("valu")) +
              "\n  " + ", ".join(f"{k} {c[k]}" for k in sorted(c) if not k.startswith("valu")))
        top = collections.Counter(i for i in ins if classify(i) in ("valu_int_addr_other", "valu_move", "valu_select_cmp"))
        print("  top non-fp VALU:", ", ".join(f"{k} {v}" for k, v in top.most_common(8)))


if __name__ == "__main__":
    main()
