set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "knn16" > gpurun_out/r10g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r10g_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r10g_tests.log | head; exit $rc; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof_r10g -o run -- python3 tools/normals_prof.py 8 > gpurun_out/r10g_normals.log 2>&1 || exit 1
grep -i "normals" $(find gpurun_out/nprof_r10g -name "*kernel_stats.csv") | cut -c1-60,100-180
timeout -k 10 300 python bench.py --workload pyramid --graphs --no-p2plane --steps 96 > gpurun_out/r10g_pyramid.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r10g_pyramid.log').read().strip().splitlines()[-1]);print('pyramid', round(d['value']), round(d['frames_per_s'],1), d['roofline']['frac'])"
TAG=r10g VARIANTS="cold6 cold8" TESTS=tests/test_gpu_batch.py bash scripts/gpu_variants.sh
