#!/bin/bash
# Round-4: the driver's 8-GPU layouts rehearsed on ONE GPU (8 gloo ranks sharing it; times are
# host-staged gloo, not a measurement): config 4 width d = 128 with --verify (every rank's
# block bit-exact vs a single-device propagation of the whole graph) on the default grid
# (F = 4 feature groups x 2 row shards), one exchange candidate (gloo times mean nothing).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --dist-backend gloo \
    --dim 128 --feature-groups 4 --exchange allgather --steps 2 --warmup 1 --verify > $OUT/harness8_d128.json 2> $OUT/harness8_d128.err
echo done
