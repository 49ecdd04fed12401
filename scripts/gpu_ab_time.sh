# same-box variant timing: AB_VARIANTS="base v1 v2" AB_CFGS="bicycle dense" bash scripts/gpu_ab_time.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${AB_CFGS:-bicycle}; do
  timeout -k 10 500 python scripts/ab_time.py $c default $AB_VARIANTS 2>&1 | tee -a gpurun_out/ab_time.log || exit 1
done
