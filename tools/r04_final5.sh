#!/bin/bash
# Round-4 final tree (placed hop tables), part 2: d = 128 profile (config 4 width, no CPU
# baseline) and the other BASELINE configs with their checks.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--dim 128" NO_CPU=1 bash tools/profile_round.sh r04final3_d128
timeout -k 10 900 python -u tools/bench_configs.py --configs 2 3 4 5 6 9 --steps 10 \
    > $OUT/final3_configs.jsonl 2> $OUT/final3_configs.err
echo done
