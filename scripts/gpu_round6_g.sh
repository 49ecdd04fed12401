# round 6: split_cells (the SplitBLAS analogue) on the trained-splat stand-in, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/ab_time.py trained default default:AB_SPLIT=5 default:AB_SPLIT=10 default:AB_SPLIT=20 default:AB_SPLIT=40 default > gpurun_out/r06/ab_split_trained.log 2>&1 || { cat gpurun_out/r06/ab_split_trained.log; exit 1; }
cat gpurun_out/r06/ab_split_trained.log
timeout -k 10 300 python -u scripts/ab_time.py bicycle default default:AB_SPLIT=10 default:AB_SPLIT=20 default > gpurun_out/r06/ab_split_bicycle.log 2>&1 || { cat gpurun_out/r06/ab_split_bicycle.log; exit 1; }
cat gpurun_out/r06/ab_split_bicycle.log
