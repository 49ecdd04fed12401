# Traversal diagnostics (STATS build counters, phase cycles) on the dense stand-in and bicycle, several K.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_traversal.py dense 16 24 32 > gpurun_out/diag_dense.json 2>&1 || { cat gpurun_out/diag_dense.json; exit 1; }
cat gpurun_out/diag_dense.json
timeout -k 10 200 python scripts/diag_traversal.py bicycle 24 32 > gpurun_out/diag_bicycle.json 2>&1 || { cat gpurun_out/diag_bicycle.json; exit 1; }
cat gpurun_out/diag_bicycle.json
