#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw7
timeout -k 10 120 tools/cu_probe > gpurun_out/sw7/cu.txt 2>&1 || exit 1
head -12 gpurun_out/sw7/cu.txt | grep -v ids
tools/sweep.sh gpurun_out/sw7 \
 ";--steps 3 --warmup 1 --reserve-cus 32" \
 ";--steps 3 --warmup 1 --reserve-cus 64" \
 ";--steps 3 --warmup 1 --reserve-cus 16"
cat gpurun_out/sw7/sweep.txt
