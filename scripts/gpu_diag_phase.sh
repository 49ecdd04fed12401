set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in bicycle dense; do
timeout -k 10 300 python scripts/diag_traversal.py $cfg 24 > gpurun_out/diag_phase_$cfg.json 2>&1 || exit 1
done
grep -A8 phase_frac gpurun_out/diag_phase_bicycle.json gpurun_out/diag_phase_dense.json
