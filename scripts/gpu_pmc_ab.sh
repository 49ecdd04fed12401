set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmcab
mkdir -p $out
for v in default n64; do
  if [ "$v" = default ]; then unset GVRT_LIB_PATH; else export GVRT_LIB_PATH=$PWD/3dgvrt_lightfield_amd/build/n64/libgvrt.so; fi
  i=0; mkdir -p $out/$v
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_render" -d $out/$v/p$i -o run --output-format csv -- python3 scripts/prof_render.py > $out/$v/p$i.log 2>&1 || { echo "pmc $v $i failed"; tail -5 $out/$v/p$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $out/$v > $out/$v/summary.json || exit 1
done
