#!/bin/bash
# Round-4 GPU call 9: config 3 (G100M NGCF K=3 + GAS) under the kernel tracer with the full
# per-dispatch trace, to see each hop's duration in sequence and the gaps between kernels
# (tools/exp_hop_context.py: a hop right after a matrix-core kernel starts ~0.3 ms slow and
# recovers over ~6 hops).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g9_c3 -o run -- \
    python3 -u tools/bench_configs.py --configs 3 --steps 10 --no-ref-check > $OUT/g9_c3.jsonl 2> $OUT/g9_c3.err
echo done
