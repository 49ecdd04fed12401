set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in default $AB_VARIANTS; do
  if [ "$v" = default ]; then unset GVRT_LIB_PATH; else export GVRT_LIB_PATH=$PWD/3dgvrt_lightfield_amd/build/$v/libgvrt.so; fi
  timeout -k 10 240 python scripts/diag_traversal.py bicycle $AB_K > gpurun_out/ab/$v.json 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab/$v.json; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v.json').read()[open('gpurun_out/ab/$v.json').read().index('{'):]); print('$v', {k:(v['ms'],v['node_visits/wave'],v['leaf_visits/wave'],v.get('accel_ms')) for k,v in d.items()})"
done
