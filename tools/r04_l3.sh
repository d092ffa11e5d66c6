#!/bin/bash
# round 4: does K3's second read of the records come from the Infinity Cache (256 MiB) when a
# launch group is small enough?  Headline workload, launch groups of 1..32 maps, K1 loads plain
# or non-temporal, one stream or two groups in flight.  Map side only (no resolve/legs).
set -o pipefail
O=gpurun_out/r04_l3; mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --resolve 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --self-check 0"
for gm in 32 4 2 1; do
  for nt in 0 -1; do
    timeout -k 10 120 $B --group-maps $gm --tuning hist_nt=$nt > $O/g${gm}_nt${nt}.json 2> $O/g${gm}_nt${nt}.err || exit 1
    timeout -k 10 120 $B --group-maps $gm --tuning hist_nt=$nt --map-pipeline 0 > $O/g${gm}_nt${nt}_s1.json 2> $O/g${gm}_nt${nt}_s1.err || exit 1
    echo "gm=$gm nt=$nt done"
  done
done
