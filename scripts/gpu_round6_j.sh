# round 6: piece-marked split leaves -- tests, then same-box timing against the previous commit (build/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_api.py tests/test_gpu_sah.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/tests_j.log 2>&1 || { tail -40 gpurun_out/r06/tests_j.log; exit 1; }
tail -3 gpurun_out/r06/tests_j.log
timeout -k 10 400 python -u scripts/ab_time.py bicycle base default default:AB_SPLIT=10 default:AB_SPLIT=10,AB_SPAN=3 base default > gpurun_out/r06/ab_split3_bicycle.log 2>&1 || { cat gpurun_out/r06/ab_split3_bicycle.log; exit 1; }
cat gpurun_out/r06/ab_split3_bicycle.log
timeout -k 10 400 python -u scripts/ab_time.py trained base default default:AB_SPLIT=10 default:AB_SPLIT=10,AB_SPAN=3 default > gpurun_out/r06/ab_split3_trained.log 2>&1 || { cat gpurun_out/r06/ab_split3_trained.log; exit 1; }
cat gpurun_out/r06/ab_split3_trained.log
for cfg in garden dense; do
timeout -k 10 400 python -u scripts/ab_time.py $cfg default default:AB_SPLIT=10 default:AB_SPLIT=10,AB_SPAN=3 default > gpurun_out/r06/ab_split3_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_split3_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_split3_$cfg.log
done
