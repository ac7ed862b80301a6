#!/bin/bash
# The round's evidence in one call: gpu_evidence.sh (tests, smoke, PMC, the
# default bench, rocprof stats, iteration profiles) then gpu_configs.sh (the
# other BASELINE configs' lines, their PMC passes) without repeating the tests.
#   TAG=r10 bash scripts/gpu_round_evidence.sh
set -o pipefail
bash scripts/gpu_evidence.sh || exit $?
SKIP_TESTS=1 bash scripts/gpu_configs.sh || exit $?
