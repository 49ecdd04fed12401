# Round 6, first GPU pass: the new robustness tests, the frame pins and SAH equality (the depth budget must leave the
# stand-ins' trees and frames unchanged), then the default bench line with its new roofline / configs fields.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_frame_digest.py "tests/test_gpu_sah.py::test_device_sah_equals_host" -x -v -s --timeout 700 --timeout-method thread > gpurun_out/r06/tests_a.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06/tests_a.log
tail -30 gpurun_out/r06/tests_a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --pmc-keep gpurun_out/r06/pmc_a > gpurun_out/r06/bench_a.json 2> gpurun_out/r06/bench_a.err
rc=$?
tail -3 gpurun_out/r06/bench_a.err
exit $rc
