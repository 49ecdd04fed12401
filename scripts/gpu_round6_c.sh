set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_app.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r06/tests_c0.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06/tests_c0.log; tail -12 gpurun_out/r06/tests_c0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u -m pytest tests/test_gpu_deep.py::test_trained_standin_vs_oracle "tests/test_gpu_parity.py::test_bicycle_full_frame_vs_oracle_and_fast_literal" tests/test_gpu_configs.py -v -s --timeout 900 --timeout-method thread > gpurun_out/r06/tests_c.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06/tests_c.log
tail -20 gpurun_out/r06/tests_c.log
exit $rc
