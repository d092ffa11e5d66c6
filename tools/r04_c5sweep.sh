#!/bin/bash
# round 4: C5 after the scan rewrite — workgroups per CU of the two passes, launch-group sizes
set -o pipefail
O=gpurun_out/r04_c5sweep; mkdir -p $O
L="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0"
run() { tag=$1; shift; timeout -k 10 200 python3 bench.py $L "$@" > $O/$tag.json 2> $O/$tag.err || exit 1; echo "$tag done"; }
run base
run wgs1 --tuning small_wgs_per_cu=1
run g100 --group-maps 100
run g400 --group-maps 400
run base2
