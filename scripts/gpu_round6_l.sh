# round 6: grid / span sweep of the large-proxy split on the four 1 M-3 M stand-ins, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for cfg in trained dense bicycle garden; do
timeout -k 10 500 python -u scripts/ab_time.py $cfg default default:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=6,AB_SPAN=2 default:AB_SPLIT=8,AB_SPAN=3 default:AB_SPLIT=12,AB_SPAN=3 default:AB_SPLIT=16,AB_SPAN=4 default:AB_SPLIT=16,AB_SPAN=3 default:AB_SPLIT=10,AB_SPAN=3 > gpurun_out/r06/ab_sweep_$cfg.log 2>&1 || { cat gpurun_out/r06/ab_sweep_$cfg.log; exit 1; }
cat gpurun_out/r06/ab_sweep_$cfg.log
done
