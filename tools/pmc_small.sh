#!/bin/bash
# One GPU call: PMC passes (profiles/collect_pmc.py) for the small-record workload with the default
# (two-level MSD) kernels, then the C5 bench line.
set -o pipefail
tag=${1:-pmc_small}; out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python3 profiles/collect_pmc.py --out $out --workload small > $out/collect.log 2>&1 || { tail -30 $out/collect.log; exit 1; }
python3 -c "import json; d=json.load(open('$out/small/summary.json')); [print(k, round(v.get('hbm_bytes_per_launch',0)/v['records_per_launch'],2), 'B/rec') for k,v in d['kernels'].items()]"
legs="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0"
timeout -k 10 300 python -u bench.py --workload small $legs > $out/bench_small.json 2> $out/bench_small.err || { tail -30 $out/bench_small.err; exit 1; }
cat $out/bench_small.json
