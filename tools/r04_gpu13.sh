#!/bin/bash
# Round-4 GPU call 13: (1) hop vs row stride (tools/exp_hop_stride.py); (2) config 5 at G1B
# (10M x 10M, 1e9 pairs, host-built operand — the form that completed this round) under the
# kernel tracer only (no counters), per profiles/r03/g1b_box_loss_record.md's plan.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/exp_hop_stride.py > $OUT/g13_hop_stride.jsonl 2> $OUT/g13_hop_stride.err
free -g > $OUT/g13_free.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g13_g1b -o run -- \
    python3 -u tools/bench_configs.py --configs 5 --g1b --host-build --steps 3 --warmup 1 --no-ref-check \
    > $OUT/g13_g1b_kt.jsonl 2> $OUT/g13_g1b_kt.err
echo done
