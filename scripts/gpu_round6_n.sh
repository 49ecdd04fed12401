# round 6: API tests (duplicate tile list); acceptance boxes for mixed nodes (build/mixed) vs default; fine-grid splits
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06/tests_n.log 2>&1 || { tail -40 gpurun_out/r06/tests_n.log; exit 1; }
tail -2 gpurun_out/r06/tests_n.log
for cfg in trained bicycle dense garden; do
timeout -k 10 400 python -u scripts/ab_time.py $cfg default:AB_SPLIT=10,AB_SPAN=3 mixed@q:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=10,AB_SPAN=3 mixed@q:AB_SPLIT=10,AB_SPAN=3 > gpurun_out/r06/ab_mixed_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_mixed_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_mixed_$cfg.log
done
for cfg in trained bicycle; do
timeout -k 10 400 python -u scripts/ab_time.py $cfg default:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=32,AB_SPAN=3 default:AB_SPLIT=64,AB_SPAN=3 default:AB_SPLIT=128,AB_SPAN=3 default:AB_SPLIT=256,AB_SPAN=4 > gpurun_out/r06/ab_fine_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_fine_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_fine_$cfg.log
done
