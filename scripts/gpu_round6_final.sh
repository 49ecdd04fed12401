# round 6: the driver's own round-end commands, as it runs them (quiet suite, then the default bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/r06/final_pytest.log 2>&1 || { tail -30 gpurun_out/r06/final_pytest.log; exit 1; }
tail -2 gpurun_out/r06/final_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r06/final_bench.json 2> gpurun_out/r06/final_bench.err || { tail -20 gpurun_out/r06/final_bench.err; exit 1; }
cut -c1-400 gpurun_out/r06/final_bench.json
