#!/bin/bash
# Round-4 final tree (placed hop tables): the whole -m gpu suite and smoke().
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ \
    > $OUT/final3_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > $OUT/final3_smoke.log 2>&1
echo done
