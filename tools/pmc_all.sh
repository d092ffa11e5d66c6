#!/bin/bash
# PMC passes (profiles/collect_pmc.py) for every workload, then a kernel-trace stats run of each
# workload's default bench line.  usage: tools/pmc_all.sh TAG [workloads...]
set -o pipefail
tag=${1:-r02}; shift
ws=("$@"); [ ${#ws[@]} -eq 0 ] && ws=(small terasort zipf)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in "${ws[@]}"; do
  echo "== pmc $w"
  timeout -k 10 600 python3 -u profiles/collect_pmc.py --out gpurun_out/pmc_$tag --workload $w \
    > gpurun_out/pmc_${tag}_$w.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}_$w.log; exit 1; }
  grep -A3 '"hbm_bytes_per_launch"' gpurun_out/pmc_${tag}_$w.log | head -20
done
