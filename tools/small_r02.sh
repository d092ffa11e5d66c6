#!/bin/bash
# C5 (16-byte records, R = 10000) map side: kernel split and the small-record scatter knobs.
set -o pipefail
out=gpurun_out/${1:-r02_small}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --workload small --no-cpu-baseline --steps 5 --warmup 2 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; k=m['kernels_ms']; s=d['steps']; print('%-16s %8.1f GB/s  ms/step %7.2f  hist %6.2f scan %6.2f scatter %6.2f  k3 frac %.3f %s check %s' % ('$name', d['value'], d['ms_per_step'], k['hist']/s, k['scan']/s, k['scatter']/s, d['roofline']['frac'], d['roofline']['kernel'], d['self_check']['ok']))"
}
run two8 --map-pipeline 0 --tuning small_kernel=3
run two16 --map-pipeline 0 --tuning small_kernel=3,small_waves=16
run two8_t16k --map-pipeline 0 --tuning small_kernel=3,tile_records=16384
run two8_g128 --map-pipeline 0 --tuning small_kernel=3 --group-maps 128
run sorted_g128 --map-pipeline 0 --group-maps 128
