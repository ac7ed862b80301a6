set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread -k "small or callers or umap or voxel" > gpurun_out/r10b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "seq sums of|passed|failed|callers' workload" gpurun_out/r10b_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_r10b -o run -- python3 tools/callers_prof.py ref 3 > gpurun_out/r10b_callers.log 2>&1 || exit 1
grep pair gpurun_out/r10b_callers.log
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_r10b -name "*kernel_trace.csv") > gpurun_out/r10b_callers_iteration_profile.txt
head -5 gpurun_out/r10b_callers_iteration_profile.txt | cut -c1-100; tail -2 gpurun_out/r10b_callers_iteration_profile.txt
TAG=r10v VARIANTS="i0w12 i0w16" bash scripts/gpu_variants.sh
