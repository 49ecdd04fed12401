# One-GPU rehearsal of bench.py's multi-GPU frame-exchange step (torch.distributed.run, one rank, RCCL):
# per-step time of the exchange path vs the plain one-GPU path, views (bicycle) and tiles (truck).
# OLD=bench_oldsync.py adds the previous (host-synchronous) exchange for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --no-pmc --no-stats"
run1() {  # name, script, config, extra
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 500)) $2 --gpus 1 --exchange --config $3 $B $4 > gpurun_out/ex_$1.log 2>&1 \
        && grep -h '^{' gpurun_out/ex_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['value'], d.get('kernel_ms'))"
}
plain() {
    timeout -k 10 240 python bench.py --config $2 $B $3 > gpurun_out/ex_$1.log 2>&1 \
        && grep -h '^{' gpurun_out/ex_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['value'], d.get('kernel_ms'))"
}
if [ -z "$ONLYOLD" ]; then plain plain_bicycle bicycle && run1 ex_bicycle bench.py bicycle && \
plain plain_truck truck "--split tiles" && run1 ex_truck bench.py truck "--split tiles"; fi && \
if [ -n "$OLD" ]; then run1 old_bicycle $OLD bicycle && run1 old_truck $OLD truck "--split tiles"; fi
