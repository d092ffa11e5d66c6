#!/bin/bash
# Round 3: can a key-only K1 fetch less than 100 B per TeraSort record?  (tools/key_probe.hip)
set -o pipefail
out=gpurun_out/keyprobe
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 ./tools/key_probe > $out/plain.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $out/pmc_fetch -o run -- ./tools/key_probe > $out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum --kernel-trace -d $out/pmc_req -o run -- ./tools/key_probe > $out/pmc_req.log 2>&1 || exit $?
cat $out/plain.txt
