# per-kernel times of the parallel sequential sums (tools/seqsum_prof.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dev}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sqprof_${TAG} -o run -- python3 tools/seqsum_prof.py > gpurun_out/${TAG}_sqprof.log 2>&1
echo "rocprof rc=$?"
cat gpurun_out/${TAG}_sqprof.log | tail -12
f=$(find gpurun_out/sqprof_${TAG} -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -20
