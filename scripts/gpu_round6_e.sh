# round 6: the whole GPU suite (parity figures land in gpurun_out/parity/), then smoke; a heartbeat file under
# gpurun_out/ shows progress while a long parity test (minutes, no output until it ends) runs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
(while sleep 50; do date +%T >> gpurun_out/r06/heartbeat.log; done) &
hb=$!
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --durations=15 --timeout 900 --timeout-method thread > gpurun_out/r06/tests_e.log 2>&1
rc=$?
kill $hb
echo "pytest rc=$rc" >> gpurun_out/r06/tests_e.log
tail -22 gpurun_out/r06/tests_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke_e.log 2>&1
rc=$?
tail -2 gpurun_out/r06/smoke_e.log
exit $rc
