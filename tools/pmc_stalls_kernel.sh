#!/bin/bash
# Stall decomposition of one kernel under any command: the two PMC passes of
# tools/pmc_stalls.sh (SQ wave-cycle buckets; TA/TD/TCP/GRBM) around "$@", each its own run.
#   bash tools/pmc_stalls_kernel.sh <out_dir> <kernel_substring> -- <python3 ...>
set -euo pipefail
OUT=$1; K=$2; shift 3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- "$@" > $OUT/sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/tc -o run -- "$@" > $OUT/tc.log 2>&1
python tools/pmc_table.py $K $(find $OUT/sq $OUT/tc -name "*counter_collection.csv") > $OUT/summary.json
cat $OUT/summary.json
