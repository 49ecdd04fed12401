# Cache-counter passes on one config's render loop: GVRT_CFG=dense [GVRT_OPTS=compact_nodes=1 GVRT_TAG=c1] bash scripts/gpu_pmc_cfg.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_${GVRT_CFG:-bicycle}${GVRT_TAG:+_$GVRT_TAG}
mkdir -p $out
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 scripts/pmc_summary.py $out > $out/pmc_summary.json && head -40 $out/pmc_summary.json
