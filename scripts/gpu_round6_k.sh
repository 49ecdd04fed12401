# round 6: the quality build with large-proxy pieces -- split / digest tests, then trained and dense vs the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_frame_digest.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r06/tests_k0.log 2>&1
echo "rc=$?" >> gpurun_out/r06/tests_k0.log
grep -E "digest|passed|failed|PASSED|FAILED" gpurun_out/r06/tests_k0.log | tail -30
timeout -k 10 1000 python -u -m pytest tests/test_gpu_deep.py::test_trained_standin_vs_oracle tests/test_gpu_configs.py::test_dense_standin tests/test_gpu_parity.py::test_bicycle_full_frame_vs_oracle_and_fast_literal -v -s --timeout 900 --timeout-method thread > gpurun_out/r06/tests_k1.log 2>&1
rc=$?
tail -5 gpurun_out/r06/tests_k1.log
exit $rc
