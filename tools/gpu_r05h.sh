set -o pipefail
O=gpurun_out/r05_h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/diag_hip.py > $O/diag.txt 2>&1; echo "diag rc=$?"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort.py > $O/sort_tests.txt 2>&1; rc=$?; echo "sort tests rc=$rc"; tail -3 $O/sort_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_random.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_partition.txt 2>&1 || exit 1
tail -1 $O/sort_random.txt $O/sort_partition.txt
L="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0"
for i in 1 2; do
timeout -k 10 200 python3 bench.py $L > $O/c5_lo4_$i.json 2> $O/c5_lo4_$i.err || exit 1
timeout -k 10 200 python3 bench.py $L --tuning msd_direct=8 > $O/c5_lo5_$i.json 2> $O/c5_lo5_$i.err || exit 1
echo "round $i done"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py -k "owned or peer_major or tickets or export_cache or single_rank" tests/test_gpu_bench_rehearsal.py > $O/own_tests.txt 2>&1; echo "own tests rc=$?"; tail -3 $O/own_tests.txt
