#!/bin/bash
# Map side on a CU-masked stream (the N > 1 configuration) at N = 1: grids sized to the mask.
set -o pipefail
out=gpurun_out/${1:-r02_reserve}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --map-pipeline 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; k=m['kernels_ms']; s=d['steps']; print('%-18s %8.1f GB/s  ms/step %7.2f  hist %6.2f scan %6.2f scatter %6.2f  check %s' % ('$name', d['value'], d['ms_per_step'], k['hist']/s, k['scan']/s, k['scatter']/s, d.get('self_check', {}).get('ok')))"
}
run all_cus
run reserve32 --reserve-cus 32
run small_reserve32 --workload small --reserve-cus 32
run rccl_at_one --rccl-at-one --self-check 0
