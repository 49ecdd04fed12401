# Traversal diagnostics (STATS counters + phase cycles): CFGS="bicycle dense" KS="24" OPTS_LIST="none octant_nodes=0"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
for cfg in ${CFGS:-bicycle}; do
  for opts in ${OPTS_LIST:-none}; do
    o=$opts; [ "$o" = none ] && o=""
    DIAG_OPTS=$o timeout -k 10 300 python scripts/diag_traversal.py $cfg ${KS:-24} > gpurun_out/diag/${cfg}_${opts//[=,]/_}.json 2> gpurun_out/diag/${cfg}_${opts//[=,]/_}.err || { tail -5 gpurun_out/diag/${cfg}_${opts//[=,]/_}.json; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/diag/${cfg}_${opts//[=,]/_}.json')); k=[x for x in d if x.startswith('fast')][0]; v=d[k]; print('$cfg', '$opts', k, v['ms'], 'nodes', v['node_visits/wave'], 'leaves', v['leaf_visits/wave'], v.get('phase_frac'))"
  done
done
