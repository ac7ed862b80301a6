#!/bin/bash
# One GPU session: tests, smoke, bench, kernel-trace profile.  Every GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"; tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"; tail -3 gpurun_out/prof.log
find gpurun_out/prof_${TAG} -name "*stats*" | head
