set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_traversal.py bicycle > gpurun_out/diag.json 2>&1; cat gpurun_out/diag.json
