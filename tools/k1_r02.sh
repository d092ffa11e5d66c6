#!/bin/bash
# K1 (k_hist4) sweep: records per LDS stage and workgroups per CU.
set -o pipefail
out=gpurun_out/${1:-r02_k1}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --map-pipeline 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; k=m['kernels_ms']; s=d['steps']; print('%-18s %8.1f GB/s  ms/step %7.2f  hist %6.2f scan %6.2f scatter %6.2f  check %s' % ('$name', d['value'], d['ms_per_step'], k['hist']/s, k['scan']/s, k['scatter']/s, d['self_check']['ok']))"
}
run h64
run h128 --tuning hist_stage=128
run h64_w2 --tuning hist_wgs_per_cu=2
run h64_w3 --tuning hist_wgs_per_cu=3
run h128_w2 --tuning hist_stage=128,hist_wgs_per_cu=2
run h64_t8k --tuning tile_records=8192
