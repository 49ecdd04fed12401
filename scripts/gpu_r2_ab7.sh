set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="comp8 comp6 default comp8 comp6" AB_CFGS="bicycle dense garden" timeout -k 10 700 bash scripts/gpu_ab_time.sh
