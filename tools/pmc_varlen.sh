#!/bin/bash
# PMC passes over the variable-length map side (bench.py varlen leg; the TeraSort part is cut to
# 1 Mi records): HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes), L2->fabric write request
# sizes, wave occupancy/stall counters.  One counter group per pass.
set -o pipefail
out=gpurun_out/pmcv; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python3 bench.py --steps 1 --warmup 1 --records 1048576 --no-cpu-baseline --reduce-sort-records 0 $*"
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"} \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $out/p$i -o run --output-format csv -- $B > $out/p$i.log 2>&1 || { tail $out/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcv/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if not any(t in k for t in os.environ.get("PMC_FILTER", "k_v").split(",")): continue
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print("==", k)
    for c, v in sorted(cs.items()):
        print("   %-26s %16.1f per dispatch (%d)" % (c, sum(v) / len(v), len(v)))
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        f = 2 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
        w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        print("   HBM bytes/launch: read %.3f GB (FETCH_SIZE x2) write %.3f GB" % (f / 1e9, w / 1e9))
PY
