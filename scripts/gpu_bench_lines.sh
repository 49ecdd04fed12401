# Several bench.py lines in one GPU call: BENCH_LINES="--config truck --rank-balance 8;--camera-path orbit" \
#   bash scripts/gpu_bench_lines.sh   -> $L/<n>.json (+ .err), one summary line each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=${BENCH_OUT:-gpurun_out}/lines; mkdir -p $L
i=0
IFS=';' read -ra LINES <<< "$BENCH_LINES"
for line in "${LINES[@]}"; do
  i=$((i+1))
  timeout -k 10 ${TLIMIT:-300} python bench.py $line > $L/$i.json 2> $L/$i.err || { echo "line $i ($line) failed"; tail -5 $L/$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$L/$i.json')); print('$i', '$line', '|', d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['kernel_ms'], 'kernel ms', 'first', d.get('first_frame_kernel_ms'), 'balance', d.get('rank_balance'))"
done
