#!/bin/bash
# Round-4 GPU call 15: the training GPU tests (incl. the one-rank tiled step into NativeAdam),
# configs 5 6 9 with their checks, then the GAT table-layout A/B (tools/exp_gat_layout.py).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_training_gpu.py > $OUT/g15_training_tests.log 2>&1
timeout -k 10 900 python -u tools/bench_configs.py --configs 5 6 9 --steps 10 \
    > $OUT/g15_configs_5_6_9.jsonl 2> $OUT/g15_configs_5_6_9.err
timeout -k 10 400 python -u tools/exp_gat_layout.py > $OUT/g15_gat_layout.jsonl 2> $OUT/g15_gat_layout.err
echo done
