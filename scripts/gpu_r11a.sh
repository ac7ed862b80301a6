#!/bin/bash
# kNN-16 leftovers by wavefront (k_normals_wave): parity + timing; cold-seed
# sparse-ring variants A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "knn16 or normals or p2plane or fpfh" > gpurun_out/r11a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11a_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r11a_tests.log | head; exit $rc; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof_r11a -o run -- python3 tools/normals_prof.py 8 > gpurun_out/r11a_normals.log 2>&1 || exit 1
grep -i "normals" $(find gpurun_out/nprof_r11a -name "*kernel_stats.csv") | cut -c1-60,100-180
TAG=r11a VARIANTS="s3 s4" bash scripts/gpu_variants.sh
