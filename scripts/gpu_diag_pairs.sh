set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in bicycle dense; do
GVRT_LIB_PATH=$GRAFT_REPO_ROOT/3dgvrt_lightfield_amd/build/diagpairs/libgvrt.so timeout -k 10 300 python scripts/diag_traversal.py $cfg 24 > gpurun_out/diag_pairs_$cfg.json 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/diag_pairs_$cfg.json'.replace('.json','.json'))) if False else None" ; tail -30 gpurun_out/diag_pairs_$cfg.json | grep -E "fast_k24|leaf_visits|dead_visits|late_node|lane_leaf|node_visits" 
done
