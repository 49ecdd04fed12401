# round 6: size-selective split (split_min_span) on the trained stand-in and bicycle, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/ab_time.py trained default default:AB_SPLIT=10 default:AB_SPLIT=10,AB_SPAN=3 default:AB_SPLIT=20,AB_SPAN=3 default:AB_SPLIT=20,AB_SPAN=5 default:AB_SPLIT=40,AB_SPAN=4 default:AB_SPLIT=40,AB_SPAN=8 default:AB_SPLIT=80,AB_SPAN=8 default > gpurun_out/r06/ab_span_trained.log 2>&1 || { cat gpurun_out/r06/ab_span_trained.log; exit 1; }
cat gpurun_out/r06/ab_span_trained.log
timeout -k 10 400 python -u scripts/ab_time.py bicycle default default:AB_SPLIT=20,AB_SPAN=3 default:AB_SPLIT=20,AB_SPAN=5 default:AB_SPLIT=40,AB_SPAN=4 default:AB_SPLIT=40,AB_SPAN=8 default > gpurun_out/r06/ab_span_bicycle.log 2>&1 || { cat gpurun_out/r06/ab_span_bicycle.log; exit 1; }
cat gpurun_out/r06/ab_span_bicycle.log
