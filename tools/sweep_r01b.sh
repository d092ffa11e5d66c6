#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw2
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw2/tests.log 2>&1 || { tail -30 gpurun_out/sw2/tests.log; exit 1; }
tail -2 gpurun_out/sw2/tests.log
tools/sweep.sh gpurun_out/sw2 \
 ";--steps 3 --warmup 1" \
 "SUX_S6=512;--steps 3 --warmup 1" \
 "SUX_S6=384;--steps 3 --warmup 1" \
 "SUX_S6=256;--steps 3 --warmup 1" \
 "SUX_S6_TPW=32;--steps 3 --warmup 1" \
 "SUX_S6_TPW=4;--steps 3 --warmup 1" \
 "SUX_S6=512 SUX_S6_TPW=16;--steps 3 --warmup 1"
cat gpurun_out/sw2/sweep.txt
