# Run a subset of the GPU tests: TESTS="tests/test_gpu_sah.py" [KEXPR="options or digest"] bash scripts/gpu_test_one.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIMIT:-500} python -u -m pytest ${TESTS} ${KEXPR:+-k "$KEXPR"} -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_one.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_one.log
tail -25 gpurun_out/pytest_one.log
exit $rc
