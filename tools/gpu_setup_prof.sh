#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/setup_prof
for c in C5 C4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/setup_prof/$c -o run -- python3 tools/setup_prof.py --cfg $c > gpurun_out/setup_prof/$c.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for c in ("C5", "C4"):
    f = glob.glob(f"gpurun_out/setup_prof/{c}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    print(c)
    for r in rows[:14]:
        print("  %-70s calls %5s total_ms %8.3f avg_us %9.1f" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 120 python -u tools/passtime.py --dims 256,256,128 --rhs 25 --op RT || exit 1
timeout -k 10 120 python -u tools/passtime.py --dims 4096,4096 --rhs 25 --op RT || exit 1
timeout -k 10 300 python -u tools/kn_phases.py --only C5,C4 || exit 1
