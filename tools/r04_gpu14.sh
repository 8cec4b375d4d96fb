#!/bin/bash
# Round-4 GPU call 14: hop-table layout A/B on the bench path (tools/exp_hop_tables.py), the
# distributed / full-size GPU tests with the placed tables, and a short bench run.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_hop_tables.py > $OUT/g14_hop_tables.jsonl 2> $OUT/g14_hop_tables.err
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_distributed_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_models_gpu.py \
    > $OUT/g14_tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vendor > $OUT/g14_bench.json 2> $OUT/g14_bench.err
echo done
