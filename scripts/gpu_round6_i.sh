# round 6: split pieces with per-leaf payloads, acceptance boxes, origin records and exact boxes: tests + same-box timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_api.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/tests_i.log 2>&1 || { tail -40 gpurun_out/r06/tests_i.log; exit 1; }
tail -3 gpurun_out/r06/tests_i.log
timeout -k 10 500 python -u scripts/ab_time.py trained default default:AB_SPLIT=5 default:AB_SPLIT=10 default:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=20,AB_SPAN=3 default:AB_SPLIT=40,AB_SPAN=8 default > gpurun_out/r06/ab_split2_trained.log 2>&1 || { cat gpurun_out/r06/ab_split2_trained.log; exit 1; }
cat gpurun_out/r06/ab_split2_trained.log
timeout -k 10 400 python -u scripts/ab_time.py bicycle default default:AB_SPLIT=10 default:AB_SPLIT=20,AB_SPAN=3 default:AB_SPLIT=40,AB_SPAN=8 default > gpurun_out/r06/ab_split2_bicycle.log 2>&1 || { cat gpurun_out/r06/ab_split2_bicycle.log; exit 1; }
cat gpurun_out/r06/ab_split2_bicycle.log
