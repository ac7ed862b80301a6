set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q -s --timeout 300 --timeout-method thread -k "small or callers or batch or voxel or umap or accum" > gpurun_out/r10c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "seq sums of|passed|failed|callers' workload" gpurun_out/r10c_tests.log | head -20; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r10c_tests.log | head; exit $rc; }
for fl in 0 1; do
  if [ $fl = 1 ]; then export RST_SMALL_FB_N=0; else unset RST_SMALL_FB_N; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_r10c_$fl -o run -- python3 tools/callers_prof.py ref 3 > gpurun_out/r10c_callers_$fl.log 2>&1 || exit 1
  grep pair gpurun_out/r10c_callers_$fl.log
  python3 scripts/iter_profile_all.py $(find gpurun_out/callers_r10c_$fl -name "*kernel_trace.csv") > gpurun_out/r10c_callers_iteration_profile_$fl.txt
  head -5 gpurun_out/r10c_callers_iteration_profile_$fl.txt | cut -c1-120; tail -2 gpurun_out/r10c_callers_iteration_profile_$fl.txt | cut -c1-400
done
unset RST_SMALL_FB_N
for lf in 16384 4096 1024; do
  RST_LANE_MIN_FLOOR=$lf timeout -k 10 120 python3 tools/callers_prof.py ref 3 > gpurun_out/r10c_floor_$lf.log 2>&1 || exit 1
  echo "floor $lf"; grep pair gpurun_out/r10c_floor_$lf.log
done
