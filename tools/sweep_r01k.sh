#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw11
tools/sweep.sh gpurun_out/sw11 \
 ";--steps 3 --warmup 1 --streams 2" \
 ";--steps 3 --warmup 1 --streams 2 --group-maps 16" \
 ";--steps 3 --warmup 1 --streams 2 --group-maps 8" \
 ";--steps 3 --warmup 1 --streams 3 --group-maps 16" \
 ";--steps 3 --warmup 1"
cat gpurun_out/sw11/sweep.txt
