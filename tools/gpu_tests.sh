#!/bin/bash
# One GPU call: the -m gpu suite (or the given test paths), stops at the first failure.
# usage: tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
tag=${1:-r02}; shift
out=gpurun_out/$tag
mkdir -p $out
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 900 python -u -m pytest "${args[@]}" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -40 $out/tests.log
exit $rc
