# PMC A/B of the CU-local dispatch (default) vs the global cost order (GVRT_CU_SCHED=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_cu
mkdir -p $out/m0 $out/m1
for mode in 1 0; do
i=0
for set in "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  i=$((i+1))
  GVRT_CU_SCHED=$mode timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/m$mode/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/m$mode/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $out/m$mode/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out/m$mode > $out/m$mode.json; echo "mode $mode"; python3 -c "import json; d=json.load(open('$out/m$mode.json')); print(json.dumps(d['per_dispatch'], indent=0))"
done
