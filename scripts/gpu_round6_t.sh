# round 6: the trained stand-in's own bench line (PMC passes: VALU issue, cache, latency) and its rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06/trained
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config trained --steps 20 --warmup 5 --no-cpu-baseline --pmc-keep gpurun_out/r06/trained > gpurun_out/r06/trained/bench.json 2> gpurun_out/r06/trained/bench.err || { tail -20 gpurun_out/r06/trained/bench.err; exit 1; }
cat gpurun_out/r06/trained/bench.json | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/trained/prof -o run --output-format csv -- python3 bench.py --config trained --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/r06/trained/bench_prof.json 2> gpurun_out/r06/trained/bench_prof.err || { tail -20 gpurun_out/r06/trained/bench_prof.err; exit 1; }
find gpurun_out/r06/trained/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r06/trained/kernel_stats.csv \;
head -3 gpurun_out/r06/trained/kernel_stats.csv | cut -c1-200
