# round 6: k-buffer depth on the trained stand-in and the others (quality build), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for cfg in trained bicycle; do
timeout -k 10 300 python -u scripts/ab_time.py $cfg default:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=10,AB_SPAN=3,AB_K=24 default:AB_SPLIT=10,AB_SPAN=3,AB_K=16 default:AB_SPLIT=10,AB_SPAN=3 > gpurun_out/r06/ab_k_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_k_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_k_$cfg.log
done
