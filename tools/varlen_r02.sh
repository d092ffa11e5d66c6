#!/bin/bash
# k_vscatter3 (varlen_kernel 3) against k_vscatter2: GPU parity of the varlen tests, then the
# bench's varlen leg (32 Mi UnsafeRow-framed rows, 1 Mi-row maps, R = 200) per kernel and tile,
# then a kernel-trace of each.
set -o pipefail
out=gpurun_out/vl3; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_varlen.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
B="python -u bench.py --records 1048576 --steps 1 --warmup 1 --no-cpu-baseline --reduce-sort-records 0"
for v in 2 3; do for t in 0 1024 4096; do
  timeout -k 10 120 $B --tuning varlen_kernel=$v,varlen_tile=$t > $out/b_${v}_${t}.json 2> $out/b_${v}_${t}.err || { tail $out/b_${v}_${t}.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/b_${v}_${t}.json').read().strip().splitlines()[-1]); print('v$v tile $t', d['varlen'])"
done; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 2 3; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof$v -o run --output-format csv -- $B --tuning varlen_kernel=$v > $out/prof$v.log 2>&1 || { tail $out/prof$v.log; exit 1; }
  f=$(find $out/prof$v -name '*kernel_stats.csv' | head -1); grep -E "k_v|Name" $f | cut -c1-160
done
