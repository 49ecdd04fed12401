# round 6: the oracle-side parity tests again (explain prefers exact alternatives), with a heartbeat
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
(while sleep 50; do date +%T >> gpurun_out/r06/heartbeat.log; done) &
hb=$!
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py::test_bicycle_full_frame_vs_oracle_and_fast_literal tests/test_gpu_configs.py tests/test_gpu_deep.py::test_trained_standin_vs_oracle tests/test_gpu_fuzz.py -v --durations=8 --timeout 900 --timeout-method thread > gpurun_out/r06/tests_q.log 2>&1
rc=$?
kill $hb
tail -14 gpurun_out/r06/tests_q.log
exit $rc
