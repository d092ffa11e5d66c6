#!/bin/bash
# round 4, final tree: a headline-only rocprof kernel trace + stats (K3's launch mean vs the
# bench's HIP-event mean), and the sort's kernel trace on range-partition keys
set -o pipefail
O=gpurun_out/r04_finalprof; mkdir -p $O
export TMPDIR=/tmp
LEGS="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_headline -o run -- python3 bench.py --steps 5 --warmup 2 $LEGS --self-check 0 > $O/prof_headline.json 2> $O/prof_headline.err || exit 1
SORT_PROF_INPUT=partition timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_sort -o run -- python3 tools/sort_prof.py 20 > $O/prof_sort.txt 2>&1
