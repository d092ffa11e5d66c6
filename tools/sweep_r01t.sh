#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw20
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw20/tests.log 2>&1 || { tail -40 gpurun_out/sw20/tests.log; exit 1; }
tail -1 gpurun_out/sw20/tests.log
timeout -k 10 120 tools/stamps > gpurun_out/sw20/stamps.txt 2>&1 || { cat gpurun_out/sw20/stamps.txt; exit 1; }
cat gpurun_out/sw20/stamps.txt
tools/sweep.sh gpurun_out/sw20 ";--steps 3 --warmup 1" ";--steps 3 --warmup 1"
cat gpurun_out/sw20/sweep.txt
