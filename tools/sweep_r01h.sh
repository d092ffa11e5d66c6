#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw8
timeout -k 10 120 tools/stamps > gpurun_out/sw8/stamps.txt 2>&1 || { cat gpurun_out/sw8/stamps.txt; exit 1; }
cat gpurun_out/sw8/stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw8/tests.log 2>&1 || { tail -30 gpurun_out/sw8/tests.log; exit 1; }
tail -2 gpurun_out/sw8/tests.log
tools/sweep.sh gpurun_out/sw8 \
 ";--steps 3 --warmup 1" \
 "SUX_SCATTER=v6;--steps 3 --warmup 1" \
 ";--steps 3 --warmup 1 --workload zipf"
cat gpurun_out/sw8/sweep.txt
