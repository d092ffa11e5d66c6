#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw4
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw4/tests.log 2>&1 || { tail -30 gpurun_out/sw4/tests.log; exit 1; }
tail -2 gpurun_out/sw4/tests.log
tools/sweep.sh gpurun_out/sw4 \
 ";--steps 3 --warmup 1" \
 ";--steps 3 --warmup 1 --group-maps 16" \
 "SUX_TILE_RECS=4096;--steps 3 --warmup 1 --group-maps 16" \
 ";--steps 3 --warmup 1 --group-maps 32"
cat gpurun_out/sw4/sweep.txt
