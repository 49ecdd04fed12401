# GPU parity tests, then a same-box A/B of the render kernel (default build vs build/<variant>/ libs).
# usage: AB_VARIANTS="base x" AB_K=24 bash scripts/gpu_check_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh
