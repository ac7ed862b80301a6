#!/bin/bash
# PMC passes on the ICP kernels (one counter group per rocprofv3 run).
export TMPDIR=/tmp
LIBSEL=${LIBSEL:-realsensetracker_amd/lib/librst_align.so}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  RST_LIB=$LIBSEL timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_icp|k_solve" --output-format csv -d gpurun_out/pmc$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-p2plane > gpurun_out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc$i.log; exit 1; }
  echo "pass $i ok"
done
