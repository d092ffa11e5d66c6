#!/bin/bash
# GPU: partitioner parity (every kind, the small-record paths, varlen), pass A alone, then the C5
# and C4 driver legs (3 steps each) — after the modulo-by-R change (mod_pos / part_magic).
set -o pipefail
O=gpurun_out/${1:-r06_fm}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_pipelined.py \
  tests/test_gpu_varlen.py -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2; do timeout -k 10 60 ./tools/msd_whatif0 >> $O/passa.jsonl || exit 1; done
cat $O/passa.jsonl
LEG="--steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 \
--reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0"
for w in small zipf; do
  timeout -k 10 400 python3 -u bench.py --workload $w $LEG > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); \
print('$w', d['value'], d['ms_per_step'], d['roofline_map_side']['kernels_ms'], d.get('self_check',{}).get('ok'))"
done
