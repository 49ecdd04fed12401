# scheduler-strategy variants of the render kernel (same source, -mllvm -amdgpu-sched-strategy=...)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="max-ilp max-memory-clause iterative-ilp default max-ilp max-memory-clause iterative-ilp" AB_CFGS="bicycle dense" timeout -k 10 800 bash scripts/gpu_ab_time.sh
