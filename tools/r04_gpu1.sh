#!/bin/bash
# Round-4 GPU call 1: the new full-size parity tests, the whole -m gpu suite, the N=1 bench with
# the vendor comparator (no CPU baseline: it is timed by the driver's default run), and the
# 2-rank gloo harness of bench.py's layout candidates (two ranks sharing the one GPU).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_fullsize_models_gpu.py > $OUT/g1_fullsize_models.log 2>&1
timeout -k 10 900 $T -m gpu tests/ --ignore=tests/test_fullsize_models_gpu.py > $OUT/g1_gpu_tests.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/g1_bench.json 2> $OUT/g1_bench.err
timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo \
    --users 200000 --items 200000 --pairs 4000000 --steps 3 --warmup 1 --verify \
    > $OUT/g1_harness2.json 2> $OUT/g1_harness2.err
echo done
