# seqsum.hip on the GPU: the bit-exact tests, the walk statistics, and the
# per-kernel times (rocprofv3 --kernel-trace --stats) of tools/seqsum_prof.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dev}
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqsum.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_seqsum_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_seqsum_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_seqsum_tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sqprof_${TAG} -o run -- python3 tools/seqsum_prof.py > gpurun_out/${TAG}_seqsum_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
grep -v "^W2026\|^I2026" gpurun_out/${TAG}_seqsum_prof.log | tail -14
f=$(find gpurun_out/sqprof_${TAG} -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-5 "$f" | head -12
exit $rc
