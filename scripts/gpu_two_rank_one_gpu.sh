# Rehearsal: can two RCCL ranks share the one GPU of this box? (native C++ split, tile and view layouts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/tworank
python3 -c "import importlib,sys; sys.path.insert(0,'.'); gv=importlib.import_module('3dgvrt_lightfield_amd'); gv.save_ply('gpurun_out/tworank/scene.ply', gv.scene.config1(n=3000))"
for layout in cost-bands views; do
  rm -f gpurun_out/tworank/id_$layout
  extra=""; [ "$layout" = "views" ] && extra="--views 16 --width 96 --height 64"
  for rank in 0 1; do
    timeout -k 5 90 ./3dgvrt_lightfield_amd/gvrt_app split --ply gpurun_out/tworank/scene.ply --rank $rank --world 2 --id-file gpurun_out/tworank/id_$layout --frames 4 --layout $layout $extra --out gpurun_out/tworank/out_${layout}_$rank > gpurun_out/tworank/${layout}_$rank.log 2>&1 &
  done
  wait
  echo "== $layout"; tail -3 gpurun_out/tworank/${layout}_0.log; tail -3 gpurun_out/tworank/${layout}_1.log
done
