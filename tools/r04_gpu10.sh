#!/bin/bash
# Round-4 GPU call 10: the config-3 layer-2 hop (tools/exp_hop_offset.py).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_hop_offset.py > $OUT/g10_hop_offset.jsonl 2> $OUT/g10_hop_offset.err
echo done
