set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest "tests/test_gpu_parity.py::test_bicycle_full_frame_vs_oracle_and_fast_literal" tests/test_gpu_configs.py::test_lightfield_grid_16_views tests/test_gpu_configs.py::test_dense_standin -v -s --timeout 900 --timeout-method thread > gpurun_out/r06/tests_d.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06/tests_d.log
tail -8 gpurun_out/r06/tests_d.log
exit 0
