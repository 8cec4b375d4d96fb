#!/bin/bash
# Round-4 GPU call 4: the quad plan layout (3 plan loads per 4 chunks instead of 12) —
# bit-exactness through the tiled tests with the variant library, then a same-box hop A/B.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
GNNREC_LIB=tools/bin/libgnnrec_quad.so timeout -k 10 900 $T tests/test_tiled_factor_gpu.py \
    tests/test_fullsize_gpu.py tests/test_long_rows_gpu.py tests/test_hop_schedule.py \
    --deselect tests/test_tiled_factor_gpu.py::test_factor_kernel_counts_mismatches > $OUT/g4_quad_tests.log 2>&1
timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g4_sweep_base.jsonl 2> $OUT/g4_sweep_base.err
GNNREC_LIB=tools/bin/libgnnrec_quad.so timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g4_sweep_quad.jsonl 2> $OUT/g4_sweep_quad.err
timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g4_sweep_base2.jsonl 2> $OUT/g4_sweep_base2.err
GNNREC_LIB=tools/bin/libgnnrec_quad.so timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g4_sweep_quad2.jsonl 2> $OUT/g4_sweep_quad2.err
GNNREC_LIB=tools/bin/libgnnrec_quad.so timeout -k 10 600 python bench.py --no-cpu-baseline --no-vendor > $OUT/g4_bench_quad.json 2> $OUT/g4_bench_quad.err
timeout -k 10 600 python bench.py --no-cpu-baseline --no-vendor > $OUT/g4_bench_base.json 2> $OUT/g4_bench_base.err
for V in t_v1 t_v3 t_v1 t_v3; do
  GNNREC_LIB=tools/bin/libgnnrec_$V.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/g5_c3_$V -o run -- python3 tools/bench_configs.py --configs 3 --steps 10 --no-ref-check \
      > $OUT/g5_c3_$V.jsonl 2> $OUT/g5_c3_$V.err
done
echo done
