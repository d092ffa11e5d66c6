#!/bin/bash
# GPU: tools/msd_whatif.hip at levels 0 / 1 / 2 (pass A alone; 2 x each, alternating), then one
# LDS-conflict PMC pass per level.  Output under gpurun_out/${1:-r06_w}/.
set -o pipefail
O=gpurun_out/${1:-r06_w}
mkdir -p $O
for i in 1 2; do
  for L in ${LEVELS:-0 1 2 a}; do
    timeout -k 10 60 ./tools/msd_whatif$L >> $O/whatif.jsonl 2>> $O/whatif.err || { echo "level $L failed"; exit 1; }
  done
done
cat $O/whatif.jsonl
for L in ${PMCLEVELS:-0 a}; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
    --output-format csv -d $O/pmc$L -o run -- ./tools/msd_whatif$L > $O/pmc$L.log 2>&1 || { echo "pmc $L failed"; exit 1; }
done
echo whatif done
