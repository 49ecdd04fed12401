set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
timeout -k 10 600 python -m pytest tests/test_gpu_split.py -x -q > gpurun_out/split/tests.log 2>&1 && \
for sc in 0 10 20; do DIAG_SPLIT=$sc timeout -k 10 240 python scripts/diag_traversal.py bicycle 24 > gpurun_out/split/diag_$sc.json 2>&1 || exit 1; done
