#!/bin/bash
# round 4: k_scatter8 image writes as 2 x ds_write2_b32 (A, default) vs four lane-rotated
# ds_write_b32 (B, SUX_K3_ROT: conflict-free where a record's units are contiguous); headline map
# side only, alternating, each line self-checked
set -o pipefail
O=gpurun_out/r04_k3rot; mkdir -p $O
B=/tmp/k3b; rm -rf $B; mkdir -p $B && cp -r bench.py sparkucx_amd profiles oracle $B/ && cp tools/ab/libB_k3rot.so $B/sparkucx_amd/libsparkucx_amd.so || exit 1
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --resolve 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0"
for i in 1 2; do
  timeout -k 10 150 python3 bench.py $ARGS >> $O/A.jsonl 2>> $O/A.err || exit 1
  (cd $B && timeout -k 10 150 python3 bench.py $ARGS) >> $O/B.jsonl 2>> $O/B.err || exit 1
done
echo done
