# Bench lines for every BASELINE.json config that fits one GPU (parity cases beside the headline workload).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
for cfg in ${CFGS:-bicycle garden truck lightfield dense}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-10} --warmup ${WARMUP:-2} --no-cpu-baseline > gpurun_out/configs/$cfg.json 2> gpurun_out/configs/$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/configs/$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/configs/$cfg.json')); print('$cfg', d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['kernel_ms'], 'kernel ms', d['roofline']['frac'], 'frac', d['enclose_ms'], d['accel_ms'], d['config']['width'], d['config']['height'], d['config']['views'], d['config']['survivors'])"
done
