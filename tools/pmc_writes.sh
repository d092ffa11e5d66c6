#!/bin/bash
# L2 -> fabric write request sizes: full 64-B requests vs others, for the run-copy probe (aligned
# and misaligned runs) and the bench's scatter.  One counter group per pass.
set -o pipefail
out=gpurun_out/pmcw
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $out/probe -o run --output-format csv -- tools/hbm_probe 4000 > $out/probe.log 2>&1 || { tail $out/probe.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $out/bench -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --records 268435456 --no-cpu-baseline --reduce-sort-records 0 > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("probe", "bench"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/pmcw/{tag}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0][:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", tag)
    for k, cs in acc.items():
        w = cs.get("TCC_EA0_WRREQ_sum", [0]); w64 = cs.get("TCC_EA0_WRREQ_64B_sum", [0])
        if sum(w) == 0: continue
        print("  %-60s dispatches %3d  wrreq/disp %12.0f  64B %5.1f%%" % (k, len(w), sum(w)/len(w), 100*sum(w64)/max(1,sum(w))))
PY
