#!/bin/bash
# Round-4 GPU call 6: NGCF with compact hop inputs (the transform stores its rows twice: the
# concat block and the next layer's compact input) — tests, the hop on a strided vs compact
# input table, config 3 timing + its torch-reference check; then the 8-rank d = 128 harness.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_real_shapes_gpu.py \
    tests/test_fullsize_models_gpu.py tests/test_tiled_plan_gpu.py tests/test_capi.py \
    tests/test_distributed_gpu.py > $OUT/g6_tests.log 2>&1
timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g6_sweep_ld64.jsonl 2> $OUT/g6_sweep_ld64.err
timeout -k 10 300 python tools/sweep_tiled.py --ldx 256 1117:49152:4096 > $OUT/g6_sweep_ld256.jsonl 2> $OUT/g6_sweep_ld256.err
timeout -k 10 600 python tools/bench_configs.py --configs 3 --steps 10 > $OUT/g6_config3.jsonl 2> $OUT/g6_config3.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g6_c3 -o run -- \
    python3 tools/bench_configs.py --configs 3 --steps 10 --no-ref-check > $OUT/g6_c3_kt.jsonl 2> $OUT/g6_c3_kt.err
bash tools/r04_harness8.sh
echo done
