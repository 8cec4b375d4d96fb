#!/bin/bash
# Round-4 GPU call 11: map of the column-block effect (tools/exp_hop_offset2.py).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_hop_offset2.py > $OUT/g11_hop_offset2.jsonl 2> $OUT/g11_hop_offset2.err
echo done
