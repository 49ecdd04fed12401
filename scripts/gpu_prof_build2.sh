# rocprofv3 kernel stats of the quality accel build (builder 2 = device binned SAH, collapse 1 = SAH-optimal DP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pb2
GVRT_B=2 GVRT_C=1 timeout -k 10 200 python scripts/prof_build.py > gpurun_out/pb2/plain.log 2>&1 || { cat gpurun_out/pb2/plain.log; exit 1; }
cat gpurun_out/pb2/plain.log
GVRT_B=2 GVRT_C=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pb2/prof -o run --output-format csv -- python3 scripts/prof_build.py > gpurun_out/pb2/prof.log 2>&1 || { tail gpurun_out/pb2/prof.log; exit 1; }
find gpurun_out/pb2/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/pb2/kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/pb2/kernel_stats.csv')))
for r in rows[:30]: print(r['Name'][:90].ljust(90), r['Calls'].rjust(6), '%10.1f us' % (float(r['TotalDurationNs'])/1e3))
"
