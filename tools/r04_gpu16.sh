#!/bin/bash
# Round-4 GPU call 16: d = 64 hop-table start offset A/B (tools/exp_hop_tables2.py).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_hop_tables2.py > $OUT/g16_hop_tables2.jsonl 2> $OUT/g16_hop_tables2.err
echo done
