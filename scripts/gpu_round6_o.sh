# round 6: the randomised parity sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r06/tests_fuzz.log 2>&1
rc=$?
grep -E "^case|PASSED|FAILED|passed|failed|Error" gpurun_out/r06/tests_fuzz.log | tail -60
exit $rc
