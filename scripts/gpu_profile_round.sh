# Full measurement pass for profiles/: GPU tests, smoke, the bench line (PMC passes + CPU baseline), rocprofv3 kernel
# stats of the same bench command, PMC passes on the render loop, every config's bench line, the moving-camera and
# rank-balance lines.  usage: TAG=r04 [SKIP_TESTS=1] [PMC_ONLY=1] [PART=1|2] bash scripts/gpu_profile_round.sh
# (PART=1: tests, smoke, bench, rocprof stats, PMC passes; PART=2: the other configs' lines and the extra lines --
# each part fits one gpurun call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/$TAG
mkdir -p $out/pmc
if [ "$PART" != "2" ]; then
if [ -z "$PMC_ONLY" ]; then
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --pmc-keep $out > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-configs > $out/bench_prof.json 2> $out/bench_prof.err || { tail -20 $out/bench_prof.err; exit 1; }
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find $out/prof -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
head -5 $out/kernel_stats.csv
# the line's figures recomputed from the kept PMC rows and the trace's launch groups (first frame / timed / later)
python3 scripts/reproduce_line.py $out/bench.json $out/bench_pmc.json $out/kernel_trace.csv --warmup 5 --steps 20 > $out/line_reproduction.json && cat $out/line_reproduction.json
fi
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/pmc/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/pmc/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 scripts/pmc_summary.py $out/pmc > $out/pmc_summary.json && head -30 $out/pmc_summary.json
[ -n "$PMC_ONLY" ] && exit 0
fi
[ "$PART" = "1" ] && exit 0
for cfg in garden truck lightfield dense; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $out/config_$cfg.json 2> $out/config_$cfg.err || { echo "$cfg failed"; tail -5 $out/config_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/config_$cfg.json')); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], d['kernel_ms'], r['bound'], r['frac'], r.get('cache', {}).get('l2_frac'), r.get('latency', {}).get('frac'), r.get('hbm', {}).get('frac'))"
done
for cfg in bicycle dense; do
  timeout -k 10 200 python3 scripts/orbit_costs_dump.py $out/orbit_costs_$cfg.npz $cfg 0.1 0.5 2 > $out/orbit_costs_$cfg.log 2>&1 || { echo "orbit costs $cfg failed"; tail -5 $out/orbit_costs_$cfg.log; exit 1; }
  cat $out/orbit_costs_$cfg.log
done
BENCH_OUT=$out BENCH_LINES="${EXTRA_LINES:---camera-path orbit --orbit-step 0.5 --steps 40 --no-pmc --no-cpu-baseline --no-stats;--camera-path orbit --orbit-step 2 --steps 40 --no-pmc --no-cpu-baseline --no-stats;--config truck --rank-balance 8 --no-pmc --no-cpu-baseline --no-stats;--config lightfield --rank-balance 8 --no-pmc --no-cpu-baseline --no-stats}" bash scripts/gpu_bench_lines.sh
