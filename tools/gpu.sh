#!/bin/bash
# One parametrised GPU-box runner.  It replaces the per-call tools/gpu_r*_*.sh one-offs of rounds
# 2-5 (the headers of older profiles/ files cite them; they are in the git history before round 6).
#
#   TAG=r6a bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the call (no
# GPU step runs after a failure, a fault or a time-limit kill).  Output: gpurun_out/${TAG}_*.
#   pytest            the whole -m gpu suite            pytest=EXPR   only tests matching -k EXPR
#   smoke             __graft_entry__.smoke()
#   bench             python bench.py (defaults)        bench=ARGS    with these arguments ('+' = space)
#   bench_trim[=ARGS] the bench with HGP_POOL_MB=1024 (idle plans trimmed: per-call re-allocation)
#   configs           tools/bench_configs.py (five-config table)
#   phases[=C2,C4]    tools/kn_phases.py --only ...
#   passtime=D/B/OP[,D/B/OP...]   tools/passtime.py --dims D --rhs B --op OP (D: 4096x4096)
#   profile           rocprofv3 --kernel-trace --stats of the bench (tools/profile.sh)
#   pmc               PMC HBM bytes of the C2 K matvec (tools/pmc_kop.sh)
#   profcfg=D/B/OP[,...]  per-kernel stats + PMC bytes of one batched op (tools/prof_cfg.sh)
#   py=SCRIPT+ARGS    any python script (timeout 600 s; log ${TAG}_py<k>.log for the k-th py step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/${TAG}

npy=0
fail() { echo "[gpu.sh] step '$1' failed (rc $2)"; [ -n "$3" ] && tail -30 "$3"; exit 1; }

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  arg=${arg//+/ }
  echo "[gpu.sh] $(date +%T) $step"
  case $name in
    pytest)
      sel=(); [ -n "$arg" ] && sel=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread "${sel[@]}" \
        > ${O}_pytest_gpu.log 2>&1 || fail "$step" $? ${O}_pytest_gpu.log
      tail -1 ${O}_pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || fail "$step" $? ${O}_smoke.log
      tail -3 ${O}_smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py $arg > ${O}_bench.json 2> ${O}_bench.err || fail "$step" $? ${O}_bench.err
      python - ${O}_bench.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4 = d.get("strong_c4", {})
print("bench:", round(d["value"]), "RHS-matvecs/s", round(d["ms_per_step"], 4), "ms/step frac", round(d["roofline"]["frac"], 3)
      if "roofline" in d else d, "| compute_kn", round(d.get("pcg_wall_clock_ms", 0), 2), "ms | C4 leg",
      c4.get("ms"), c4.get("phase_median_ms"), c4.get("plan_scratch_bytes"), c4.get("error"))
EOF
      ;;
    bench_trim)
      # the config-4 leg with the idle-plan pool forced to trim (HGP_POOL_MB=1024): every call
      # re-allocates the plan's scratch, as round 5's 62 GB C4 plan did under the 1/8 budget
      HGP_POOL_MB=1024 timeout -k 10 600 python bench.py --no-cpu-baseline $arg > ${O}_bench_trim.json 2> ${O}_bench_trim.err \
        || fail "$step" $? ${O}_bench_trim.err
      python -c "import json,sys; d=json.loads(open('${O}_bench_trim.json').read().strip().splitlines()[-1]); print('trimmed pool C4 leg:', json.dumps(d.get('strong_c4')))" ;;
    configs)
      timeout -k 10 900 python tools/bench_configs.py > ${O}_configs.jsonl 2> ${O}_configs.err || fail "$step" $? ${O}_configs.err
      cat ${O}_configs.jsonl ;;
    phases)
      timeout -k 10 600 python tools/kn_phases.py --only ${arg:-C2,C3,C4,C5} > ${O}_kn_phases.jsonl 2> ${O}_kn_phases.err \
        || fail "$step" $? ${O}_kn_phases.err
      cat ${O}_kn_phases.jsonl ;;
    passtime)
      for spec in ${arg//,/ }; do
        IFS=/ read -r dims rhs op <<< "$spec"
        timeout -k 10 240 python tools/passtime.py --dims ${dims//x/,} --rhs $rhs --op $op >> ${O}_passtime.txt 2> ${O}_passtime.err \
          || fail "$step ($spec)" $? ${O}_passtime.err
      done
      cat ${O}_passtime.txt ;;
    profile)
      bash tools/profile.sh ${TAG} || fail "$step" $? ;;
    profcfg)
      # per-kernel stats + PMC HBM bytes of one batched operator: profcfg=4096x4096/25/RT[,...]
      for spec in ${arg//,/ }; do
        IFS=/ read -r dims rhs op <<< "$spec"
        SHAPE=${dims//x/,} RHS=$rhs OP=$op TAG=${TAG}_${dims}_${op} bash tools/prof_cfg.sh > ${O}_profcfg_${dims}_${op}.txt 2>&1 \
          || fail "$step ($spec)" $? ${O}_profcfg_${dims}_${op}.txt
        tail -25 ${O}_profcfg_${dims}_${op}.txt
      done ;;
    pmc)
      bash tools/pmc_kop.sh > ${O}_pmc_kop.log 2>&1 || fail "$step" $? ${O}_pmc_kop.log
      grep traffic_bytes_per_op gpurun_out/pmc_kop/pmc_kop_C2.json ;;
    py)
      npy=$((npy + 1))
      timeout -k 10 600 python -u $arg > ${O}_py${npy}.log 2>&1 || fail "$step" $? ${O}_py${npy}.log
      tail -40 ${O}_py${npy}.log ;;
    *)
      echo "[gpu.sh] unknown step '$step'"; exit 2 ;;
  esac
done
echo "[gpu.sh] $(date +%T) done"
