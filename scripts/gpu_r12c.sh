#!/bin/bash
# single REF aligns' fallback grid (RST_FB_BLOCKS_REF): suite, host API, callers, sharded
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r12c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r12c_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r12c_tests.log | head -20; exit $rc; }
for fb in 384 1536 2048; do
  RST_FB_BLOCKS_REF=$fb timeout -k 10 200 python tools/host_api_prof.py > gpurun_out/r12c_host_$fb.log 2>&1 || exit 1
  RST_FB_BLOCKS_REF=$fb timeout -k 10 200 python tools/callers_prof.py ref 4 > gpurun_out/r12c_callers_$fb.log 2>&1 || exit 1
  echo "fb $fb host: $(grep pair gpurun_out/r12c_host_$fb.log | sed 's/pair [0-9]: //' | tr '\n' ' ') callers: $(grep pair gpurun_out/r12c_callers_$fb.log | tail -3 | sed 's/.*total //' | tr '\n' ' ')"
done
