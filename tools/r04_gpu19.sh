#!/bin/bash
# Round-4 GPU call 19: rows per block on the bench path with placed tables.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/exp_rows_per_block.py > $OUT/g19_rows.jsonl 2> $OUT/g19_rows.err
echo done
