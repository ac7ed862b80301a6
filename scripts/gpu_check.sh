# GPU parity suite + the driver's exact bench command: a round-trip check
#   TAG=r10a [FIRST=tests/test_gpu_batch.py] bash scripts/gpu_check.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-dev}
if [ -n "$FIRST" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1
  rc=$?; echo "first rc=$rc"; tail -4 gpurun_out/${TAG}_first.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_first.log | head -20; exit $rc; }
fi
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log | cut -c1-1500
exit $rc
