#!/bin/bash
# Round 3 GPU session driver: numbered steps, each under its own time limit; stops at the first
# step that crashed or timed out (rc >= 124), records every rc.  usage: tools/r03_run.sh TAG STEP...
#   STEP = t:<pytest args>   (python -u -m pytest ... -x -v --timeout 300; shell-quoted, eval'd)
#        = b:<bench args>    (python bench.py ... > TAG/bench_N.json)
#        = p:<rocprof args>  (rocprofv3 --kernel-trace --stats -d TAG/prof_N -o run -- python bench.py ...)
#        = s:<shell>         (anything else, e.g. make)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for st in "$@"; do
  n=$((n+1))
  kind=${st%%:*}; arg=${st#*:}
  case $kind in
    t) eval "timeout -k 10 900 python -u -m pytest $arg -x -v --timeout 150 --timeout-method thread" > $out/tests_$n.log 2>&1; rc=$?
       tail -3 $out/tests_$n.log ;;
    b) timeout -k 10 600 python -u bench.py $arg > $out/bench_$n.json 2> $out/bench_$n.err; rc=$?
       cat $out/bench_$n.json | head -c 600; echo ;;
    p) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof_$n -o run --output-format csv -- python -u bench.py $arg > $out/prof_$n.json 2> $out/prof_$n.err; rc=$? ;;
    s) timeout -k 10 600 bash -c "$arg" > $out/step_$n.log 2>&1; rc=$? ;;
  esac
  echo "step $n ($kind) rc=$rc: $arg" | tee -a $out/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping: step $n crashed or timed out"; exit $rc; fi
done
exit 0
