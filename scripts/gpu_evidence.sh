#!/bin/bash
# Round evidence on one GPU: parity tests, smoke, the default bench (CPU
# baseline included), rocprof kernel stats of the same command, FETCH /
# WRITE PMC passes, a one-pair iteration trace and the fallback anatomy.
#   TAG=r02o bash scripts/gpu_evidence.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-r02}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 gpurun_out/${TAG}_$name.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
SHORT="--steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0"
PMCB="--steps 6 --warmup 1 --batch 8 --inflight 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0"
[ -n "$SKIP_TESTS" ] || step pytest_gpu 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# the PMC passes first, so that the bench line below carries this build's
# traffic (bench.py reads profiles/pmc_*.json; the copy stays on the box)
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG} -o run -- python3 bench.py $PMCB
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG} -o run -- python3 bench.py $PMCB
python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}.json $(find gpurun_out/pmcf_${TAG} -name "*counter_collection.csv") $(find gpurun_out/pmcw_${TAG} -name "*counter_collection.csv") RefAcc 8
cp gpurun_out/pmc_${TAG}.json profiles/pmc_${TAG}.json
# (gpurun copies back at most 64 MiB of gpurun_out: the raw counter and
# trace CSVs go once their summaries are written)
rm -rf gpurun_out/pmcf_${TAG} gpurun_out/pmcw_${TAG}
step bench 600 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py
python3 scripts/profile_summary.py $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv") gpurun_out/${TAG}_prof.log > gpurun_out/${TAG}_profile_summary.txt
find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" -delete
step iter 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG} -o run -- python3 bench.py --batch 0 --inflight 1 $SHORT --steps 3
python3 scripts/iter_profile_all.py $(find gpurun_out/iter_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_iteration_profile.txt
rm -rf gpurun_out/iter_${TAG}
step diag 200 env RST_LIB=realsensetracker_amd/lib/variants/diag.so python tools/diag_fb.py
# the reference callers' workload (~15k-point clouds), every kernel per iteration
step callers 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_${TAG} -o run -- python3 tools/callers_prof.py ref 3
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_callers_iteration_profile.txt
rm -rf gpurun_out/callers_${TAG}
cp gpurun_out/${TAG}_callers.log gpurun_out/${TAG}_callers_pairs.txt
