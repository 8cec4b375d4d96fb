#!/bin/bash
# Round-4 final tree: the whole -m gpu suite, smoke(), then the round profile of the headline
# (bench with the CPU baseline and the vendor comparator, rocprofv3 kernel stats, FETCH/WRITE/L2
# PMC passes) — all on the final kernel source (kernel_key).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ \
    > $OUT/final_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > $OUT/final_smoke.log 2>&1
bash tools/profile_round.sh r04final
echo done
