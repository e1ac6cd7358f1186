"""Co-residency sweep (GPU box): the batched K op (and others) timed by tools/passtime.py in fresh
processes under different minimum-LDS requests of the 2-D column conv / row kernels
(HGP_CONV_LDS_MIN, HGP_ROWF_LDS_MIN, HGP_ROWI_LDS_MIN; hgp_pass_dispatch.hpp), which cap how
many blocks of one kind a CU takes so that the two RHS streams' passes can share CUs -- or any other
environment knob of the plan (B: HGP_BALANCED_CHUNKS, S: HGP_STREAMS, W: HGP_WS_MB, P: HGP_CONV_P32, R: HGP_LR).  A case
"phases:C3,C4" runs tools/kn_phases.py (compute_kn set-up / PCG / R^T) instead of passtime.

    python tools/lds_sweep.py [--cases "4096x4096/25/K;..."] [--settings "-;C=54000;C=54000,F=80000"]
Each setting runs as a child process (this process never touches the GPU)."""
import argparse
import json
import os
import subprocess
import sys

KEYS = {"C": "HGP_CONV_LDS_MIN", "F": "HGP_ROWF_LDS_MIN", "I": "HGP_ROWI_LDS_MIN",
        "B": "HGP_BALANCED_CHUNKS", "S": "HGP_STREAMS", "W": "HGP_WS_MB", "L": "HGP_LIB",
        "P": "HGP_CONV_P32", "R": "HGP_LR"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="4096x4096/25/K;4096x4096/25/CINV;2048x2048/200/K;1024x1024/32/K")
    ap.add_argument("--settings", default="-;C=41000;C=54000;C=81000;I=41000;C=54000,I=54000")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = [c for c in a.cases.split(";") if c]
    settings = a.settings.split(";")

    def env_of(setting):
        env = dict(os.environ)
        for kv in ([] if setting.strip() in ("", "-", "base") else setting.split(",")):
            k, v = kv.split("=")
            env[KEYS[k.strip()]] = v.strip()
        return env

    # settings interleaved per case and repetition (A B A B ...), so a drift of the box's clock
    # over the sweep does not masquerade as a difference between settings
    for case in cases:
        for rep in range(a.reps):
            for setting in settings:
                env = env_of(setting)
                if case.startswith("phases:"):       # compute_kn phase split (tools/kn_phases.py)
                    r = subprocess.run([sys.executable, os.path.join(root, "tools", "kn_phases.py"), "--only",
                                        case.split(":", 1)[1]], env=env, capture_output=True, text=True, timeout=600)
                    for line in r.stdout.strip().splitlines():
                        if line.startswith("{"):
                            print(json.dumps({"setting": setting, "case": case, "rep": rep, **json.loads(line)}), flush=True)
                    if r.returncode != 0:
                        print(json.dumps({"setting": setting, "case": case, "error": r.stderr[-400:]}), flush=True)
                        sys.exit(r.returncode)
                    continue
                dims, rhs, op = case.split("/")
                dims = dims.replace("x", ",")
                r = subprocess.run([sys.executable, os.path.join(root, "tools", "passtime.py"), "--dims", dims,
                                    "--rhs", rhs, "--op", op], env=env, capture_output=True, text=True, timeout=300)
                line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
                try:
                    d = json.loads(line)
                except ValueError:
                    print(json.dumps({"setting": setting, "case": case, "error": r.stderr[-400:]}), flush=True)
                    if r.returncode not in (0, 1):
                        sys.exit(r.returncode)
                    continue
                print(json.dumps({"setting": setting, "case": case, "rep": rep, "op_ms": d["op_ms"],
                                  "passes_ms": d["passes_ms"], "frac": d.get("frac")}), flush=True)


if __name__ == "__main__":
    main()
