#!/bin/bash
# Batched value leg, development loop: the sequential-sum and batch tests,
# a (pairs per batch, batches in flight) sweep, and the kernel stats of one
# batch in flight.   TAG=x CFGS="8 3|8 4" bash scripts/gpu_dev_batch.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-dbatch}
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1 --no-host-api"
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_seqsum.py tests/test_gpu_batch.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
IFS="|"
for cfg in ${CFGS:-8 3|8 4|12 3}; do
  IFS=" "; set -- $cfg
  timeout -k 10 300 python bench.py $B --batch $1 --inflight $2 --steps ${STEPS:-96} > gpurun_out/${TAG}_b$1_i$2.log 2>&1 || { tail -5 gpurun_out/${TAG}_b$1_i$2.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_b$1_i$2.log').read().strip().splitlines()[-1]);print('batch $1 inflight $2 value', round(d['value']), 'ok', d['pairs_ok'])"
  IFS="|"
done
IFS=" "
if [ -n "${PROF:-1}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py $B --batch ${PB:-8} --inflight 1 --steps 48 > /dev/null 2>&1 || exit 1
  python3 - <<PY
import csv, glob, re
f = glob.glob("gpurun_out/prof_${TAG}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    n = re.sub(r"\(.*", "", r["Name"].replace("rst::(anonymous namespace)::", ""))
    print(f"{n[:60]:<60} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
fi
