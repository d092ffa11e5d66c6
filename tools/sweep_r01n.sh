#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw14
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw14/tests.log 2>&1 || { tail -40 gpurun_out/sw14/tests.log; exit 1; }
tail -2 gpurun_out/sw14/tests.log
SUX_S7=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread -k "terasort or ragged or golden or hash or zipf" > gpurun_out/sw14/tests2.log 2>&1 || { tail -40 gpurun_out/sw14/tests2.log; exit 1; }
tail -2 gpurun_out/sw14/tests2.log
SUX_S7=2 timeout -k 10 120 tools/stamps > gpurun_out/sw14/stamps.txt 2>&1 || { cat gpurun_out/sw14/stamps.txt; exit 1; }
cat gpurun_out/sw14/stamps.txt
tools/sweep.sh gpurun_out/sw14 \
 ";--steps 3 --warmup 1" \
 "SUX_S7=2;--steps 3 --warmup 1" \
 "SUX_S7=3;--steps 3 --warmup 1"
cat gpurun_out/sw14/sweep.txt
