# round 4 GPU call K: packed-fp32 build vs the shipped one -- compute_kn phases at C2..C5; pk + 6
# waves/SIMD for the mixed-radix axis-0 convolutions (HGP_MINW_CONTIG_TRI=6: 3 blocks per CU); the
# issue / LDS / instruction-cache counters of the C2 K op's passes (what bounds them once the VALU
# instruction count drops 40 %).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PK=$PWD/hipgp_amd/libhipgp_pk.so
for lib in base pk; do
  if [ $lib = pk ]; then export HGP_LIB=$PK; else unset HGP_LIB; fi
  echo "lib $lib"
  timeout -k 10 300 python tools/kn_phases.py --only C2,C3,C4,C5 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_k.txt || exit 1
for lib in pk pkt6; do
  export HGP_LIB=$PWD/hipgp_amd/libhipgp_$lib.so
  for cfg in "4096,4096 25" "2048,2048 200" "1024,1024 32"; do
    set -- $cfg
    echo -n "$lib "; timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pkt6_k.txt || exit 1
for lib in base pk; do
  if [ $lib = pk ]; then export HGP_LIB=$PK; else unset HGP_LIB; fi
  OUT=gpurun_out/pmc_k_$lib; rm -rf $OUT; mkdir -p $OUT
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES" \
             "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
      python3 tools/passtime.py --dims 1024,1024 --rhs 32 --op K --op-only 5 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed ($lib)"; tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
done
echo done
