#!/bin/bash
# Round-4 GPU call 12: NGCF concat table placed off the slow gather line (gather_table):
# the NGCF / distributed / full-size model tests, config 3 timed with its torch-reference
# check, then config 3 under the kernel tracer (per-layer hop durations).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_models_gpu.py tests/test_fullsize_models_gpu.py tests/test_real_shapes_gpu.py \
    tests/test_distributed_gpu.py > $OUT/g12_tests.log 2>&1
timeout -k 10 600 python -u tools/bench_configs.py --configs 3 --steps 10 > $OUT/g12_config3.jsonl 2> $OUT/g12_config3.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g12_c3 -o run -- \
    python3 -u tools/bench_configs.py --configs 3 --steps 10 --no-ref-check > $OUT/g12_c3_kt.jsonl 2> $OUT/g12_c3_kt.err
echo done
