set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="tcg default tcg" AB_CFGS="bicycle dense garden" timeout -k 10 600 bash scripts/gpu_ab_time.sh
