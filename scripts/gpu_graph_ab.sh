#!/bin/bash
# hipGraph A/B: graph parity test, then stream and pyramid benches with and
# without --graphs (no CPU baseline / extra modes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "hipgraph or pyramid" --timeout 120 --timeout-method thread > gpurun_out/graph_pytest.log 2>&1 || { tail -30 gpurun_out/graph_pytest.log; exit 1; }
tail -1 gpurun_out/graph_pytest.log
for wl in stream pyramid; do
  for gf in "" "--graphs"; do
    f=gpurun_out/graph_ab_${wl}${gf}.log
    timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-p2plane --no-host-api --no-gicp $gf > $f 2>&1 || exit $?
    echo "$wl $gf: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps")')"
  done
done
