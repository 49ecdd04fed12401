# rocprofv3 kernel stats of the render loop (scripts/prof_render.py: bench scene, N renders)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pr
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pr/prof -o run --output-format csv -- python3 scripts/prof_render.py > gpurun_out/pr/prof.log 2>&1 || { tail gpurun_out/pr/prof.log; exit 1; }
find gpurun_out/pr/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/pr/kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/pr/kernel_stats.csv')))
for r in rows[:8]: print(r['Name'][:70].ljust(70), r['Calls'].rjust(6), '%10.1f us avg' % (float(r['AverageNs'])/1e3))
"
