#!/bin/bash
# Round-4 multi-rank rehearsals with the placed hop tables, on ONE GPU (gloo ranks sharing it;
# times are not a measurement): 2 ranks, every layout and candidate (default grid = 2 feature
# groups x 1 row shard: each rank runs the one-rank path on placed d = 32 tables), --verify;
# then 4 ranks at full size, d = 64 (2 x 2 grid), --verify.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --dist-backend gloo \
    --users 200000 --items 200000 --pairs 4000000 --steps 3 --warmup 1 --verify \
    > $OUT/harness2_placed.json 2> $OUT/harness2_placed.err
timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29525 bench.py --gpus 4 --dist-backend gloo \
    --exchange allgather --steps 2 --warmup 1 --verify --no-vendor \
    > $OUT/harness4_placed.json 2> $OUT/harness4_placed.err
echo done
