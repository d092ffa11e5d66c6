#!/bin/bash
# One parameterised GPU job runner (replaces the per-round r0x_*.sh / *_r02.sh scripts).
# Every GPU step runs under its own time limit; the script stops at the first failing step.
#
#   tools/gpujob.sh TAG JOB [args...]        output under gpurun_out/TAG/
#
# JOB:
#   tests [pytest args]     the -m gpu suite (or the given paths), stops at the first failure
#   smoke                   __graft_entry__.smoke()
#   bench [bench args]      bench.py (default: the driver's N = 1 line) -> bench.json
#   final                   tests + smoke + default bench (a round checkpoint)
#   trace [bench args]      rocprofv3 --kernel-trace --stats of a headline-only bench run
#   pmc WORKLOAD...         profiles/collect_pmc.py passes (one counter group per rocprofv3 run)
#   sortpmc                 PMC passes of tools/sort_prof.py (5 M TeraSort records)
#   sorttrace [N] [INPUT]   rocprofv3 kernel trace of tools/sort_prof.py (INPUT: partition (default),
#                           random, long)
#   msdprobe                kernel trace + FETCH/WRITE_SIZE passes of tools/sort_msd_probe.py
#   sortprof                the sort tests, then tools/sort_prof.py on random and range-partition keys, 2 x
#   sortab LIB_A LIB_B      tools/sort_prof.py on both inputs, A and B alternating, 2 x each
#   ab LIB_B [bench args]   bench.py alternating with a copy of the tree linking LIB_B, 2 x each
#   cmd SECONDS CMD...      any other command under a time limit
set -o pipefail
tag=${1:?usage: tools/gpujob.sh TAG JOB [args...]}; job=${2:?job}; shift 2
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
LEGS="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 \
--plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0 --no-cpu-baseline"

run_tests() {
  local a=("$@"); [ ${#a[@]} -eq 0 ] && a=(tests -m gpu)
  timeout -k 10 1500 python -u -m pytest "${a[@]}" -x -v --timeout 300 --timeout-method thread \
    > $O/tests.txt 2>&1; local rc=$?
  tail -5 $O/tests.txt; echo "tests rc=$rc"; return $rc
}
run_smoke() {
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
    && echo smoke ok
}
run_bench() {
  timeout -k 10 900 python3 -u bench.py "$@" > $O/bench.json 2> $O/bench.err; local rc=$?
  echo "bench rc=$rc"; tail -c 600 $O/bench.json; return $rc
}

case $job in
  tests) run_tests "$@" ;;
  smoke) run_smoke ;;
  bench) run_bench "$@" ;;
  final) run_tests && run_smoke && run_bench ;;
  trace)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
      python3 bench.py --steps 5 --warmup 2 $LEGS --self-check 0 "$@" > $O/prof.json 2> $O/prof.err
    ;;
  pmc)
    for w in "$@"; do
      timeout -k 10 600 python3 -u profiles/collect_pmc.py --out $O --workload $w > $O/$w.log 2>&1 \
        || { tail -5 $O/$w.log; exit 1; }
    done ;;
  sortpmc)
    i=0
    for cs in "FETCH_SIZE" "WRITE_SIZE" \
        "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
        "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
      timeout -s KILL 90 rocprofv3 --pmc $cs --output-format csv -d $O/pass$i -o run -- \
        python3 tools/sort_prof.py 5 > $O/pass$i.log 2>&1 || exit 1
      i=$((i+1))
    done ;;
  sorttrace)
    SORT_PROF_INPUT=${2:-partition} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof_sort -o run -- python3 tools/sort_prof.py ${1:-20} > $O/prof_sort.txt 2>&1 ;;
  msdprobe)
    # tools/sort_msd_probe.py (record-moving MSD first pass vs today's sort): kernel trace, then
    # one PMC pass each for FETCH_SIZE and WRITE_SIZE
    cd /tmp || exit 1
    R=$GRAFT_REPO_ROOT; [ -n "$R" ] || R=/root/repo
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
      python3 $R/tools/sort_msd_probe.py > $R/$O/probe_trace.jsonl 2> $R/$O/probe_trace.err || exit 1
    i=0
    for cs in "FETCH_SIZE" "WRITE_SIZE"; do
      timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $R/$O/pass$i -o run -- \
        python3 $R/tools/sort_msd_probe.py > $R/$O/pass$i.log 2>&1 || exit 1
      i=$((i+1))
    done; echo msdprobe done ;;
  sortprof)
    run_tests tests/test_gpu_sort.py || exit 1
    for i in 1 2; do
      timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_random_$i.txt 2>&1 || exit 1
      SORT_PROF_INPUT=partition timeout -k 10 120 python3 tools/sort_prof.py 20 \
        > $O/sort_partition_$i.txt 2>&1 || exit 1
    done
    tail -qn 1 $O/sort_random_*.txt $O/sort_partition_*.txt ;;
  sortab)
    for i in 1 2; do
      for lib in "$1" "$2"; do
        for inp in random partition ${SORTAB_EXTRA:-}; do
          SORT_PROF_INPUT=$inp timeout -k 10 120 python3 tools/sort_prof.py 20 "" $lib \
            >> $O/sortab.txt 2>&1 || exit 1
        done
      done
    done
    grep "per call" $O/sortab.txt ;;
  ab)
    lib=${1:?LIB_B}; shift
    B=/tmp/ab_b; rm -rf $B; mkdir -p $B && cp -r bench.py sparkucx_amd profiles oracle $B/ \
      && cp $lib $B/sparkucx_amd/libsparkucx_amd.so || exit 1
    for i in 1 2; do
      timeout -k 10 300 python3 bench.py "$@" >> $O/A.jsonl 2>> $O/A.err || exit 1
      (cd $B && timeout -k 10 300 python3 bench.py "$@") >> $O/B.jsonl 2>> $O/B.err || exit 1
    done; echo ab done ;;
  cmd)
    s=${1:?seconds}; shift
    timeout -k 10 $s "$@" ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
