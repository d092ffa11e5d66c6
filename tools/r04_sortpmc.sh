#!/bin/bash
# round 4: PMC of the sort (5 M random TeraSort records, tools/sort_prof.py): HBM bytes per kernel
# (FETCH_SIZE, doubled per the gfx950 rule, and WRITE_SIZE) and the texture path's stall share.
# One counter group per rocprofv3 run (rocprofv3 does not split passes).
set -o pipefail
O=gpurun_out/r04_sortpmc; mkdir -p $O
export TMPDIR=/tmp
i=0
for cs in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  timeout -s KILL 90 rocprofv3 --pmc $cs --output-format csv -d $O/pass$i -o run -- python3 tools/sort_prof.py 5 > $O/pass$i.log 2>&1 || exit 1
  i=$((i+1))
done
echo done
