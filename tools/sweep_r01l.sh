#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw12
timeout -k 10 120 tools/stamps > gpurun_out/sw12/stamps.txt 2>&1 || { cat gpurun_out/sw12/stamps.txt; exit 1; }
cat gpurun_out/sw12/stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw12/tests.log 2>&1 || { tail -30 gpurun_out/sw12/tests.log; exit 1; }
tail -2 gpurun_out/sw12/tests.log
tools/sweep.sh gpurun_out/sw12 \
 ";--steps 3 --warmup 1" \
 "SUX_S6_TPW=1;--steps 3 --warmup 1" \
 "SUX_S6_TPW=4;--steps 3 --warmup 1" \
 ";--steps 3 --warmup 1 --streams 2"
cat gpurun_out/sw12/sweep.txt
