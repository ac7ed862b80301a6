#!/bin/bash
# PMC counter passes (one run each) over scripts/diag_icp.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_WAVES;TA_TA_BUSY,TA_FLAT_READ_WAVEFRONTS,TCP_TCC_READ_REQ,TCP_PENDING_STALL_CYCLES,TCP_TCC_READ_REQ_LATENCY,GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"}
i=0
IFS=';' read -ra PS <<< "$PASSES"
for ctrs in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d gpurun_out/${TAG}_$i -o run -- python3 scripts/diag_icp.py > gpurun_out/${TAG}_$i.log 2>&1 || exit $?
done
