#!/bin/bash
# A/B kernel timing of two library builds (RST_LIB selects the .so)
export TMPDIR=/tmp
for v in A B; do
  if [ $v = A ]; then L=realsensetracker_amd/lib/librst_align.so; else L=realsensetracker_amd/lib/alt/librst_align_B.so; fi
  RST_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-p2plane > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v rc=$?"
done
