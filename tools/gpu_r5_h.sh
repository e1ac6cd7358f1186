# round 5 GPU call H: (1) C4 K op against the 2-D workspace budget (RHS per chunk: spectrum
# re-reads) and the stream count; (2) the C4 R^T conv-write question of round 4 (10.9 vs 17.7 GB
# per op between a 3-op and a 10-op PMC run): the same PMC summary with 3 and 10 ops, graphs on
# and off; (3) the headline evidence: kop-only kernel stats of the bench and the C2 K op's PMC bytes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ns in 2 1; do
  for ws in 1024 4096 16384; do
    HGP_STREAMS=$ns HGP_WS_MB=$ws timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op K 2>/dev/null | sed "s/^/streams$ns ws$ws /" || exit 1
  done
done | tee gpurun_out/r5h_c4_ws.txt
for gr in 1 0; do
  for n in 3 10; do
    HGP_GRAPH=$gr SHAPE=4096,4096 RHS=25 TAG=C4RT_g${gr}_n$n OP=RT NOPS=$n bash tools/prof_cfg.sh > gpurun_out/r5h_C4RT_g${gr}_n$n.txt 2>&1 || { tail -5 gpurun_out/r5h_C4RT_g${gr}_n$n.txt; exit 1; }
    grep -E "k_pass<float, 6144|traffic_over" gpurun_out/r5h_C4RT_g${gr}_n$n.txt | sed "s/^/graph$gr nops$n /"
  done
done
BENCH_ARGS="--kop-only --steps 50 --warmup 5" bash tools/profile.sh kop || exit 1
bash tools/pmc_kop.sh > gpurun_out/pmc_kop.log 2>&1 || { tail -20 gpurun_out/pmc_kop.log; exit 1; }
grep traffic_bytes_per_op gpurun_out/pmc_kop/pmc_kop_C2.json
