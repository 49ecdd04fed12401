# Round 6: the full-frame parity tests with every differing flagged ray explained by the oracle's alternatives,
# the ADAPTIVE kernel at the default depth, and the C++ app's split (SplitFrame over the RCCL backend) at world 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "adaptive" tests/test_gpu_app.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r06/tests_b0.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06/tests_b0.log
tail -25 gpurun_out/r06/tests_b0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_deep.py::test_trained_standin_vs_oracle "tests/test_gpu_parity.py::test_bicycle_full_frame_vs_oracle_and_fast_literal" tests/test_gpu_configs.py -v -s --timeout 900 --timeout-method thread > gpurun_out/r06/tests_b.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06/tests_b.log
tail -40 gpurun_out/r06/tests_b.log
exit $rc
