#!/bin/bash
# Round-4 closing check on the final tree: the whole -m gpu suite, smoke(), one bench line.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ \
    > $OUT/final6_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > $OUT/final6_smoke.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/final6_bench.json 2> $OUT/final6_bench.err
echo done
