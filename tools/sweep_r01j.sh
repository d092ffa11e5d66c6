#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw10
tools/sweep.sh gpurun_out/sw10 \
 ";--steps 3 --warmup 1" \
 "SUX_NT=1;--steps 3 --warmup 1" \
 "SUX_NT=2;--steps 3 --warmup 1" \
 "SUX_NT=3;--steps 3 --warmup 1"
cat gpurun_out/sw10/sweep.txt
