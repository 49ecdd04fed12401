# round 6: leaf lane utilisation and dead node visits of the trained stand-in vs bicycle (quality build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in trained bicycle; do
timeout -k 10 300 python -u scripts/ab_time.py $cfg default default:AB_SPLIT=10,AB_SPAN=3 > gpurun_out/r06/ab_util_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_util_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_util_$cfg.log
done
