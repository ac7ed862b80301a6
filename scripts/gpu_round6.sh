#!/bin/bash
# Round 6 closing evidence in one call: the GPU suite on the build and a
# value A/B against the previous commit's library (lib/variants/prev.so),
# then scripts/gpu_evidence.sh (smoke, PMC, the driver's bench, rocprof
# stats, a lone pair's iteration profile, the callers' profile).
#   TAG=r19 bash scripts/gpu_round6.sh
set -o pipefail
T=${TAG:-r19}
TAG=${T}ab TEST_DEFAULT=1 NO_VARIANT_TESTS=1 VARIANTS="prev" TESTS="tests/" bash scripts/gpu_variant_ab.sh || exit $?
SKIP_TESTS=1 TAG=$T bash scripts/gpu_evidence.sh
