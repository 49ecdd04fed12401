# round 6: the dense stand-in's own bench line (PMC passes) and its rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06/dense
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config dense --steps 20 --warmup 5 --no-cpu-baseline --pmc-keep gpurun_out/r06/dense > gpurun_out/r06/dense/bench.json 2> gpurun_out/r06/dense/bench.err || { tail -20 gpurun_out/r06/dense/bench.err; exit 1; }
cat gpurun_out/r06/dense/bench.json | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/dense/prof -o run --output-format csv -- python3 bench.py --config dense --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/r06/dense/bench_prof.json 2> gpurun_out/r06/dense/bench_prof.err || { tail -20 gpurun_out/r06/dense/bench_prof.err; exit 1; }
find gpurun_out/r06/dense/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r06/dense/kernel_stats.csv \;
head -3 gpurun_out/r06/dense/kernel_stats.csv | cut -c1-200
