#!/bin/bash
# round 4: where the bench's reduce_sort (a real reduce partition) spends its time
set -o pipefail
O=gpurun_out/r04_sortpart2; mkdir -p $O
export TMPDIR=/tmp
SORT_PROF_INPUT=partition timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_bench -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --resolve 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --self-check 0 > $O/bench.json 2> $O/bench.err
