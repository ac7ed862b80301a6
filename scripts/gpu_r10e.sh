set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "normal or knn or fpfh" > gpurun_out/r10e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r10e_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r10e_tests.log | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r10e -o run -- python3 bench.py --mode p2plane --no-host-api --no-gicp --no-cpu > gpurun_out/r10e_p2plane.log 2>&1 || exit 1
python3 scripts/profile_summary.py $(find gpurun_out/prof_r10e -name "*kernel_stats.csv") gpurun_out/r10e_p2plane.log | grep -E "normals|k_icp" | head
timeout -k 10 300 python bench.py --steps 6 --warmup 5 --no-cpu --no-host-api --no-gicp --no-p2plane > gpurun_out/r10e_bench48.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r10e_bench48.log').read().strip().splitlines()[-1]);print('48 pairs value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']))"
