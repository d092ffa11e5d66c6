#!/bin/bash
# round 4: the bogus-handle test, the --rccl-at-one kernel trace (comm stream gaps between the
# all-gather and the all-to-all), then PMC passes for zipf, terasort and small
set -o pipefail
O=gpurun_out/r04_e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_ipc_reuse.py > $O/ipc_tests.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_rccl1 -o run -- python3 bench.py --rccl-at-one --records 268435456 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err &&
bash tools/r04_pmc.sh zipf terasort small
