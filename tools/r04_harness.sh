#!/bin/bash
# Round-4 multi-rank rehearsals on ONE GPU (gloo ranks sharing it; times are host-staged gloo,
# not a measurement): 2 ranks with every layout and exchange candidate (the driver's N = 2
# path through bench.py), then 8 ranks at d = 128 on the default F = 4 x 2 grid, --verify.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --dist-backend gloo \
    --users 200000 --items 200000 --pairs 4000000 --steps 3 --warmup 1 --verify \
    > $OUT/harness2_final.json 2> $OUT/harness2_final.err
bash tools/r04_harness8.sh
echo done
