#!/bin/bash
# a lone pair's k_icp_nn wave clocks (iterations 16, 64) and the host API
# pair's kernels per iteration
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for it in 16 64; do
  RST_LIB=$PWD/realsensetracker_amd/lib/variants/nnclk$it.so timeout -k 10 120 python tools/nn_clock.py > gpurun_out/r18a_clk$it.txt 2>&1 || { tail -5 gpurun_out/r18a_clk$it.txt; exit 1; }
  cat gpurun_out/r18a_clk$it.txt
done
timeout -k 10 120 python tools/host_prof.py 3 > gpurun_out/r18a_host.txt 2>&1 || { tail -5 gpurun_out/r18a_host.txt; exit 1; }
cat gpurun_out/r18a_host.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/host_r18a -o run -- python3 tools/host_prof.py 2 > gpurun_out/r18a_hostprof.log 2>&1 || { tail -5 gpurun_out/r18a_hostprof.log; exit 1; }
python3 scripts/iter_profile_all.py $(find gpurun_out/host_r18a -name "*kernel_trace.csv") > gpurun_out/r18a_host_iteration_profile.txt
rm -rf gpurun_out/host_r18a
cut -c1-220 gpurun_out/r18a_host_iteration_profile.txt
