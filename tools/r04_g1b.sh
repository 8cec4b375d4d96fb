#!/bin/bash
# Round-4 config 5 at full size (profiles/r03/g1b_box_loss_record.md): first a 5M x 5M,
# 250M-pair power-law run (device-built operand, max degree ~1.5M); only if it completes,
# the 10M x 10M, 1B-pair G1B run with the host-built operand (the form round 2 completed),
# no profiler. Every phase line (host RSS, device memory) goes to the .err file as it happens.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
free -g > $OUT/g1b_free.txt
timeout -k 10 420 python -u tools/bench_configs.py --configs 5 --c5-shape 5000000 5000000 250000000 \
    --steps 5 --warmup 1 > $OUT/c5_g250m.jsonl 2> $OUT/c5_g250m.err
timeout -k 10 720 python -u tools/bench_configs.py --configs 5 --g1b --host-build \
    --steps 5 --warmup 1 > $OUT/c5_g1b.jsonl 2> $OUT/c5_g1b.err
echo done
