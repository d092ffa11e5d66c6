#!/bin/bash
# round 4: exchange tests after the all-to-all pieces change, then PMC for zipf/terasort/small
set -o pipefail
O=gpurun_out/r04_g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py tests/test_gpu_exchange_maps.py tests/test_gpu_bench_rehearsal.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_rccl1 -o run -- python3 bench.py --rccl-at-one --records 268435456 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err &&
bash tools/r04_pmc.sh zipf terasort
