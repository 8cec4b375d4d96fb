#!/bin/bash
# Round-4 GPU call 2: register-A NGCF transform (tests + config-3 A/B vs the round-3 kernel),
# the N=1 bench with the vendor comparator, and the 2-rank gloo harness of bench.py's layout
# candidates (two ranks sharing the one GPU).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_real_shapes_gpu.py \
    tests/test_fullsize_models_gpu.py tests/test_sparse_src_gpu.py tests/test_distributed_gpu.py \
    > $OUT/g2_tests.log 2>&1
timeout -k 10 600 python tools/bench_configs.py --configs 3 --steps 10 > $OUT/g2_config3_new.jsonl 2> $OUT/g2_config3_new.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g2_c3new -o run -- \
    python3 tools/bench_configs.py --configs 3 --steps 10 --no-ref-check > $OUT/g2_c3new_kt.jsonl 2> $OUT/g2_c3new_kt.err
GNNREC_LIB=tools/bin/libgnnrec_r03transform.so timeout -k 10 600 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/g2_c3old -o run -- \
    python3 tools/bench_configs.py --configs 3 --steps 10 --no-ref-check > $OUT/g2_c3old_kt.jsonl 2> $OUT/g2_c3old_kt.err
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/g2_bench.json 2> $OUT/g2_bench.err
timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo \
    --users 200000 --items 200000 --pairs 4000000 --steps 3 --warmup 1 --verify \
    > $OUT/g2_harness2.json 2> $OUT/g2_harness2.err
echo done
