#!/bin/bash
# Stall decomposition of the column-ordered hop (G100M d=64, one plan shape): two rocprofv3
# PMC passes (SQ wave-cycle buckets; TA/TD/TCP busy and stall counters) over
# tools/sweep_tiled.py, each its own run (MI355X_MICROARCH.md § rocprofv3 PMC slots); a
# third pass for the LDS (bank conflicts, busy) and the instruction counts. GNNREC_LIB picks
# the library (a tools/build_variant.sh variant).
set -euo pipefail
OUT=${PMC_OUT:-gpurun_out/pmc_stalls}
SW="${SWEEP_ARGS:-1117:49152:4096}"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- python3 tools/sweep_tiled.py $SW > $OUT/sq.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tc -o run -- python3 tools/sweep_tiled.py $SW > $OUT/tc.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o run -- python3 tools/sweep_tiled.py $SW > $OUT/lds.log 2>&1
python tools/pmc_table.py tiled_hop_kernel $(find $OUT/sq $OUT/tc $OUT/lds -name "*counter_collection.csv") > $OUT/summary.json
cat $OUT/summary.json
