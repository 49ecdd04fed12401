# Cache-level PMC passes for k_render (scalar cache, L2, vector L1): one counter group per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_cache
mkdir -p $out
i=0
for set in "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/p$i.log 2>&1 || { echo "pmc pass $i ($set) failed"; tail -3 $out/p$i.log; }
done
python3 scripts/pmc_summary.py $out > $out/summary.json; python3 -c "import json; d=json.load(open('$out/summary.json')); print(json.dumps(d['per_dispatch'], indent=0))"
