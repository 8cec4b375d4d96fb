#!/bin/bash
# Round-4: the bench line as the driver runs it (defaults: CPU baseline and vendor included)
# on the final bench.py.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $OUT/final7_bench.json 2> $OUT/final7_bench.err
echo done
