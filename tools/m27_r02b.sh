#!/bin/bash
# One GPU call: parity of the over-8-GiB launch group, then 2^27-record maps vs 2^20.
set -o pipefail
out=gpurun_out/m27b; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -m gpu -x -q --timeout 300 --timeout-method thread -k "8_gib or pipelined_matches or tuning_shapes" > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
legs="--varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --reduce-sort-records 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --map-records 134217728 --group-maps 1 $legs > $out/m27.json 2> $out/m27.err || { tail -20 $out/m27.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $legs > $out/m20.json 2> $out/m20.err || { tail -20 $out/m20.err; exit 1; }
python3 -c "
import json
for f in ['m27','m20']:
    d=json.load(open('$out/'+f+'.json')); r=d['roofline_map_side']; print(f, d['value'], d['ms_per_step'], {k: round(v/d['steps'],1) for k,v in r['kernels_ms'].items()}, d['self_check']['ok'])"
