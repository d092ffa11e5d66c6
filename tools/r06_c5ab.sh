#!/bin/bash
# GPU: C5's driver leg (pipelined, 3 steps) at msd_direct A and B, alternating, 2 x each.
set -o pipefail
O=gpurun_out/${1:-r06_ab}; A=${2:-24}; B=${3:-88}
mkdir -p $O
LEG="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 \
--file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 \
--c4-steps 0 --c5-steps 0"
for i in 1 2; do
  for t in $A $B; do
    timeout -k 10 300 python3 -u bench.py $LEG --tuning msd_direct=$t > $O/c5_${t}_$i.json 2>> $O/c5.err \
      || { echo "msd_direct=$t failed"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5_${t}_$i.json').read().strip().splitlines()[-1]); \
rm=d['roofline_map_side']; print('msd_direct=$t', d['value'], d['ms_per_step'], rm['kernels_ms'], d.get('self_check',{}).get('ok'))" \
      | tee -a $O/summary.txt
  done
done
