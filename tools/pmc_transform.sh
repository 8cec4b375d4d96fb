#!/bin/bash
# MFMA utilisation of the config-3 NGCF+GAS streaming transform: one PMC pass
# (3 SQ + 1 GRBM counters), kernel trace off, over tools/bench_configs.py config 3.
# usage: bash tools/pmc_transform.sh <tag>
set -euo pipefail
OUT=gpurun_out/pmc_transform_${1:-r04}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_configs.py --configs 3 --steps 3 --warmup 1 \
    --no-ref-check > $OUT/bench.jsonl 2> $OUT/bench.err
echo done
