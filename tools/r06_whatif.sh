#!/bin/bash
# GPU: C5's map side (serial launch groups, so each pass's time is its own) with the product
# library and the tools/msd_whatif.sh builds, alternating, 2 x each; prints pass A / B ms per step.
set -o pipefail
O=gpurun_out/${1:-r06_w}
mkdir -p $O
LEG="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 \
--file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 \
--c4-steps 0 --c5-steps 0 --map-pipeline 0"
for v in 1 2; do
  B=/tmp/whatif$v; rm -rf $B; mkdir -p $B && cp -r bench.py sparkucx_amd profiles oracle $B/ \
    && cp tools/whatif$v/libsparkucx_amd.so $B/sparkucx_amd/libsparkucx_amd.so || exit 1
done
for i in 1 2; do
  for v in 0 1 2; do
    d=.; [ $v -gt 0 ] && d=/tmp/whatif$v
    chk=""; [ $v -gt 0 ] && chk="--self-check 0"
    (cd $d && timeout -k 10 300 python3 -u bench.py $LEG $chk) > $O/w${v}_$i.json 2> $O/w${v}_$i.err \
      || { echo "variant $v failed"; tail -5 $O/w${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/w${v}_$i.json').read().strip().splitlines()[-1]); \
rm=d['roofline_map_side']; k=rm['kernels_ms']; n=d['steps']; \
print('whatif=$v', d['value'], d['ms_per_step'], 'passA/step', round(k['hist']/n,3), 'passB/step', round(k['scatter']/n,3))" \
      | tee -a $O/summary.txt
  done
done
