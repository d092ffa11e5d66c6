#!/bin/bash
# round 4: the sort on one range partition's keys (the bench's reduce_sort shape) vs random keys:
# timing and kernel traces of both
set -o pipefail
O=gpurun_out/r04_sortpart; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 60 python3 tools/sort_prof.py 30 sort_msd=3 >> $O/timing.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/prof_rand -o run -- python3 tools/sort_prof.py 20 > $O/prof_rand.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 120 rocprofv3 --kernel-trace -d $O/prof_part -o run -- python3 tools/sort_prof.py 20 > $O/prof_part.txt 2>&1
