# round 6: the dense stand-in's parity in two tests of every 4th ray
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
(while sleep 50; do date +%T >> gpurun_out/r06/heartbeat.log; done) &
hb=$!
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k dense -v --durations=4 --timeout 500 --timeout-method thread > gpurun_out/r06/tests_r.log 2>&1
rc=$?
kill $hb
tail -10 gpurun_out/r06/tests_r.log
exit $rc
