#!/bin/bash
# LZ4 compressor: hash-table bits x workloads (TeraSort map outputs, UnsafeRow rows).
set -o pipefail
out=gpurun_out/slz; mkdir -p $out
for hb in 10 11 12; do
  SUX_LZ4_HB=$hb timeout -k 10 120 python -u bench.py --records 33554432 --steps 1 --warmup 1 \
    --no-cpu-baseline --reduce-sort-records 0 > $out/b_$hb.json 2> $out/b_$hb.err || exit 1
  python -c "import json; d=json.loads(open('$out/b_$hb.json').read().strip().splitlines()[-1]); print('hb $hb tera', d['compress'], 'rows', d['varlen']['compress'])"
done
