#!/bin/bash
# Variable-length map side: kernel versions x tile sizes, 32 Mi UnsafeRow-framed rows, R=200.
set -o pipefail
out=gpurun_out/svl; mkdir -p $out
for v in 1 2; do for t in 0 512 1024 2048 4096; do
  SUX_VARLEN=$v SUX_VTILE=$t timeout -k 10 120 python -u bench.py --records 1048576 --steps 1 --warmup 1 \
    --no-cpu-baseline --reduce-sort-records 0 > $out/b_${v}_${t}.json 2> $out/b_${v}_${t}.err || exit 1
  python -c "import json; d=json.loads(open('$out/b_${v}_${t}.json').read().strip().splitlines()[-1]); print('v$v tile $t', d['varlen'])"
done; done
