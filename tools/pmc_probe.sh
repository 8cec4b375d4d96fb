#!/bin/bash
# TA/TD/TCP counters of the gather probe (tools/gather_probe2.hip) on one table size: what the
# per-CU data path looks like when random 128-B lines stream at the probe's rate.
#   bash tools/pmc_probe.sh <table_MiB> <out_dir>
set -euo pipefail
MB=$1; OUT=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tc -o run -- tools/bin/gather_probe2 $MB > $OUT/probe.log 2>&1
for k in "probe<4, 8>" "probe<16, 8>" "probe<8, 16>"; do
  echo "== $k"; python tools/pmc_table.py "$k" $(find $OUT/tc -name "*counter_collection.csv")
done
cat $OUT/probe.log
