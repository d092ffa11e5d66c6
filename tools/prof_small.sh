#!/bin/bash
# rocprofv3 kernel trace of the C5 bench line with the given tuning. usage: tools/prof_small.sh TAG TUNING
set -o pipefail
tag=$1; tn=$2
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --workload small --no-cpu-baseline --steps 3 --warmup 1 --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --self-check 0 --map-pipeline 0 --tuning "$tn" > $out/prof.json 2> $out/prof.err || { tail -20 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
cut -d, -f1-8 $out/kernel_stats.csv | head -12
