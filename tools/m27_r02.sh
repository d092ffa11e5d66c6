#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r02_m27}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --map-pipeline 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; k=m['kernels_ms']; l=m['launches']; s=d['steps']; print('%-14s %8.1f GB/s  ms/step %7.2f  hist %6.2f scan %6.2f scatter %6.2f launches %d  k3 avg %.3f ms check %s' % ('$name', d['value'], d['ms_per_step'], k['hist']/s, k['scan']/s, k['scatter']/s, l['scatter'], d['roofline']['avg_launch_ms'], d['self_check']['ok']))"
}
run m27_r199 --map-records 134217728 --partitions 199
run m20_r199 --partitions 199
run m27_r200_maps2 --map-records 134217728 --group-maps 2
run m25 --map-records 33554432
run m23 --map-records 8388608
