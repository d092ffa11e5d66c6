#!/bin/bash
# One GPU call: TeraSort bench at several launch-group sizes (maps of 2^20 records per group).
set -o pipefail
out=gpurun_out/groups_r02; mkdir -p $out
legs="--varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --reduce-sort-records 0 --no-cpu-baseline"
for gm in 16 24 32 48 64; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --group-maps $gm $legs > $out/g$gm.json 2> $out/g$gm.err || { tail -20 $out/g$gm.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/g$gm.json')); print('group_maps=$gm', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['self_check']['ok'])"
done
