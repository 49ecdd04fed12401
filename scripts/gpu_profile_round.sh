# Full measurement pass for profiles/: GPU tests, bench (with CPU baseline), rocprofv3 kernel stats of
# the same bench command, PMC passes (one counter group per run).  usage: TAG=v8 bash scripts/gpu_profile_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/$TAG
mkdir -p $out/pmc
if [ -z "$PMC_ONLY" ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err || { tail -20 $out/bench_prof.err; exit 1; }
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
head -5 $out/kernel_stats.csv
fi
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/pmc/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/pmc/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out/pmc > $out/pmc_summary.json && head -30 $out/pmc_summary.json
