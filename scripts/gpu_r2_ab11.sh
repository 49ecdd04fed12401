set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="base nopk default base nopk" AB_CFGS="bicycle dense" timeout -k 10 800 bash scripts/gpu_ab_time.sh
