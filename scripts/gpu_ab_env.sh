# Same-box A/B over environment settings: AB_ENVS="name1:VAR=v,VAR2=w name2:VAR=x" bash scripts/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for spec in $AB_ENVS; do
  name=${spec%%:*}; vars=${spec#*:}
  ( [ "$vars" != "$name" ] && for kv in ${vars//,/ }; do export "$kv"; done
    timeout -k 10 240 python scripts/diag_traversal.py ${AB_CFG:-bicycle} ${AB_K:-24} > gpurun_out/ab/$name.json 2>&1 ) || { echo "variant $name failed"; tail -5 gpurun_out/ab/$name.json; exit 1; }
  python3 -c "import json; t=open('gpurun_out/ab/$name.json').read(); d=json.loads(t[t.index('{'):]); print('$name', {k:(v['ms'],v['node_visits/wave'],v['leaf_visits/wave'],v.get('accel_ms')) for k,v in d.items()})"
done
