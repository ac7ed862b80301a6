# the sequential-sum kernels one at a time (tools/seqsum_stage.py), stopping
# at the first failure
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-dev}
CASE=${CASE:-alternating}
for st in 1 3 7; do
  timeout -k 10 120 python -u tools/seqsum_stage.py $st $CASE > gpurun_out/${TAG}_stage$st.log 2>&1
  rc=$?; echo "stages $st rc=$rc"; cat gpurun_out/${TAG}_stage$st.log | tail -12
  [ $rc -eq 0 ] || exit $rc
  grep -q "status 0, failed stage 0" gpurun_out/${TAG}_stage$st.log || exit 3
done
