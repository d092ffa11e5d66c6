#!/bin/bash
# GPU: msd16 parity (incl. msd_direct bit 7), pass A alone (product vs tag match, 3 x each), then
# the C5 driver leg at msd_direct 24 vs 152 (tools/r06_c5ab.sh).
set -o pipefail
O=gpurun_out/${1:-r06_tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipelined.py -k "msd16" -x -q --timeout 200 \
  --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2 3; do
  timeout -k 10 60 ./tools/msd_whatif0 >> $O/w.jsonl && timeout -k 10 60 ./tools/msd_whatift >> $O/w.jsonl || exit 1
done
cat $O/w.jsonl
bash tools/r06_c5ab.sh ${1:-r06_tag} 24 152
