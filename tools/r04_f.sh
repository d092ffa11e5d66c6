#!/bin/bash
set -o pipefail
O=gpurun_out/r04_f; mkdir -p $O
B="python3 bench.py --rccl-at-one --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 $B --records 67108864 --exchange-one-call > $O/one.json 2> $O/one.err; echo "one-call rc=$?"
timeout -k 10 200 $B --records 33554432 --group-maps 16 > $O/g16.json 2> $O/g16.err; echo "16-map groups rc=$?"
timeout -k 10 200 $B --records 50331648 --group-maps 24 > $O/g24.json 2> $O/g24.err; echo "24-map groups rc=$?"
