#!/bin/bash
# round 4: pass A with the LDS-DMA prefetch (msd_direct=4): parity, then C5 lines against the default
set -o pipefail
O=gpurun_out/r04_d; mkdir -p $O
LEGS="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipelined.py -k "msd16" > $O/msd_tests.txt 2>&1 &&
for t in 0 4 0 4; do
  timeout -k 10 240 python -u bench.py --workload small --steps 5 --warmup 2 $LEGS --tuning msd_direct=$t >> $O/c5_ab.jsonl 2>> $O/c5_ab.err || exit 1
done &&
for t in 0 4; do
  timeout -k 10 240 python -u bench.py --workload small --map-records 65536 --steps 5 --warmup 2 $LEGS --tuning msd_direct=$t >> $O/c5_m64k_ab.jsonl 2>> $O/c5_m64k_ab.err || exit 1
done
