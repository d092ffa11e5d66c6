#!/bin/bash
# usage: tools/sweep.sh OUTDIR "ENV=V ENV2=V2;bench args" ...  — stops at the first failure
out=$1; shift
mkdir -p $out
i=0
for a in "$@"; do
  i=$((i+1))
  envs="${a%%;*}"; bargs="${a#*;}"
  echo "== [$envs] $bargs" >> $out/sweep.txt
  timeout -k 10 300 env $envs python -u bench.py --no-cpu-baseline $bargs > $out/run$i.json 2> $out/run$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc" >> $out/sweep.txt; exit 1; fi
  python -c "import json; d=json.load(open('$out/run$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline_map_side']['kernels_ms'])" >> $out/sweep.txt
done
