# device SAH build: equality tests vs the host restatement + kernel profile of the build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="tests/test_gpu_sah.py" TLIMIT=300 bash scripts/gpu_test_one.sh || exit 1
GVRT_B=2 GVRT_C=1 GVRT_N=3 bash scripts/gpu_prof_build.sh
