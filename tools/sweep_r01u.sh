#!/bin/bash
# group size / stream sweep of the default three-kernel map side (TeraSort 100 GB, R=200)
set -o pipefail
out=gpurun_out/sw_u; mkdir -p $out
common="--no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --steps 5 --warmup 2"
for cfg in "--group-maps 32" "--group-maps 48" "--group-maps 64" "--group-maps 32 --streams 2" "--group-maps 64 --streams 2" "--group-maps 16 --streams 2"; do
  timeout -k 10 200 python -u bench.py $cfg $common > $out/b.json 2> $out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_map_side']['kernels_ms'])" | tee -a $out/sweep.txt
done
