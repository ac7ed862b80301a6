#!/bin/bash
# Which GPU test leaves the process aborting at exit?
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu -k "not sharded and not device_resident and not frame_prepare" > gpurun_out/diag1.log 2>&1; echo "no-torch-tests rc=$?"
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu -k "device_resident or frame_prepare" > gpurun_out/diag2.log 2>&1; echo "torch-tests rc=$?"
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu -k "sharded" > gpurun_out/diag3.log 2>&1; echo "sharded rc=$?"
tail -3 gpurun_out/diag*.log
