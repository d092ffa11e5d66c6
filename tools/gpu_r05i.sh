set -o pipefail
O=gpurun_out/r05_i; mkdir -p $O
export TMPDIR=/tmp
echo skip-tests
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u profiles/collect_pmc.py --out $O/pmc --workload small > $O/pmc_small.log 2>&1; echo "pmc rc=$?"
