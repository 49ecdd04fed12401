# first 9 of the 12 SH float4 summed before the accept branch (spill-free since the LDS-address fold)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS="sh9 default sh9 default sh9" AB_CFGS="bicycle dense garden" timeout -k 10 800 bash scripts/gpu_ab_time.sh
