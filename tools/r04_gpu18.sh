#!/bin/bash
# Round-4 GPU call 18: plan-shape re-sweep of the G100M d = 64 hop on a placed table
# (ld 128 floats: the layout hop_table gives d = 64), baseline shape first and last.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/sweep_tiled.py --ldx 128 1117:49152:4096 977:49152:4096 1042:49152:4096 \
    1160:49152:4096 1202:49152:4096 1117:40960:4096 1117:57344:4096 1117:49152:2048 1117:49152:8192 \
    1117:49152:4096 > $OUT/g18_sweep_ld128.jsonl 2> $OUT/g18_sweep_ld128.err
echo done
