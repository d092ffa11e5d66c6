#!/bin/bash
# K3: v7 (every completed 16-byte unit) against v8 (whole 128-byte lines, carried partial lines).
set -o pipefail
out=gpurun_out/${1:-r02_k3}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; k=m['kernels_ms']; s=d['steps']; print('%-18s %8.1f GB/s  ms/step %7.2f  hist %6.2f scan %6.2f scatter %6.2f  k3 %.3f %s check %s' % ('$name', d['value'], d['ms_per_step'], k['hist']/s, k['scan']/s, k['scatter']/s, d['roofline']['frac'], d['roofline']['kernel'], d['self_check']['ok']))"
}
run v8 --map-pipeline 0
run v8_tpi32 --map-pipeline 0 --tuning tiles_per_item=32
run v8_pipe --map-pipeline 1
run v8_zipf --map-pipeline 1 --workload zipf
run v8_m27 --map-pipeline 1 --map-records 134217728
