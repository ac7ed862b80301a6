set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "knn16 or normals or batch or p2plane or fpfh" > gpurun_out/r10h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r10h_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r10h_tests.log | head; exit $rc; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof_r10h -o run -- python3 tools/normals_prof.py 8 > gpurun_out/r10h_normals.log 2>&1 || exit 1
grep -i "normals" $(find gpurun_out/nprof_r10h -name "*kernel_stats.csv") | cut -c1-60,100-180
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-host-api --no-gicp > gpurun_out/r10h_bench.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r10h_bench.log').read().strip().splitlines()[-1]);print('value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), round(d['p2plane']['frames_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']), round(d['p2plane']['knn16_normals']['frames_per_s']))"
