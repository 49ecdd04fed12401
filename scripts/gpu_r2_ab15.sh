# per-lane LDS addresses folded (lane laundered per access) + term_cut formed at use: no scratch in the FAST kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_frame_digest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
AB_VARIANTS="base default base default" AB_CFGS="bicycle dense garden" timeout -k 10 800 bash scripts/gpu_ab_time.sh
