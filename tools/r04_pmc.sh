#!/bin/bash
# round 4: PMC passes (profiles/collect_pmc.py) for terasort, zipf and small -> gpurun_out/r04_pmc
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_pmc; mkdir -p $O
for w in "$@"; do
  timeout -k 10 560 python3 -u profiles/collect_pmc.py --out $O --workload $w > $O/$w.log 2>&1 || { tail -5 $O/$w.log; exit 1; }
done
