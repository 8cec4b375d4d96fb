#!/bin/bash
# Round-4 GPU call 17: L2 counters per channel for the slow gather line (exp_hop_offset_pmc.py).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT TCC_MISS --output-format csv -d $OUT/g17_pmc -o run -- \
    python3 -u tools/exp_hop_offset_pmc.py > $OUT/g17_pmc.log 2> $OUT/g17_pmc.err
echo done
