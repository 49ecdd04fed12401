# iterative-ilp scheduler vs the default, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="iterative-ilp default iterative-ilp default iterative-ilp" AB_CFGS="bicycle garden dense" timeout -k 10 800 bash scripts/gpu_ab_time.sh
