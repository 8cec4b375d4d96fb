#!/bin/bash
# Round-4: 977 rows per block — tiled / full-size GPU tests, then the d = 64 and d = 128 round
# profiles (bench, kernel stats, keyed PMC passes; no CPU baseline).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py \
    tests/test_tiled_factor_gpu.py tests/test_training_gpu.py > $OUT/final8_tests.log 2>&1
NO_CPU=1 bash tools/profile_round.sh r04final8
BENCH_ARGS="--dim 128" NO_CPU=1 bash tools/profile_round.sh r04final8_d128
echo done
