#!/bin/bash
# Round-4 GPU call 3: the whole -m gpu suite on the new transform (8 waves, double-buffered B,
# interleaved chains) and the SPW-generic tiled kernel; config-3 kernel trace; the d = 128
# plan-walk A/B (one walk per slice vs one per slice pair, same box).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/ > $OUT/g3_gpu_tests.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g3_c3 -o run -- \
    python3 tools/bench_configs.py --configs 3 --steps 10 > $OUT/g3_c3_kt.jsonl 2> $OUT/g3_c3_kt.err
timeout -k 10 300 python tools/exp_spw.py --max-rows 1279 > $OUT/g3_spw1.json 2> $OUT/g3_spw1.err
GNNREC_LIB=tools/bin/libgnnrec_spw1_ga1.so timeout -k 10 300 python tools/exp_spw.py --max-rows 1279 > $OUT/g3_spw1_ga1.json 2> $OUT/g3_spw1_ga1.err
GNNREC_LIB=tools/bin/libgnnrec_spw2.so timeout -k 10 300 python tools/exp_spw.py --max-rows 600 > $OUT/g3_spw2.json 2> $OUT/g3_spw2.err
timeout -k 10 300 python tools/exp_spw.py --max-rows 1279 > $OUT/g3_spw1_again.json 2> $OUT/g3_spw1_again.err
for V in t_dpp t_nodpp; do
  GNNREC_LIB=tools/bin/libgnnrec_$V.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/g3_c3_$V -o run -- python3 tools/bench_configs.py --configs 3 --steps 10 \
      > $OUT/g3_c3_$V.jsonl 2> $OUT/g3_c3_$V.err
done
GNNREC_LIB=tools/bin/libgnnrec_t_dpp.so timeout -k 10 600 python -u -m pytest -x -v --timeout 600 \
    --timeout-method thread tests/test_kernels_gpu.py tests/test_real_shapes_gpu.py \
    tests/test_fullsize_models_gpu.py -k "ngcf or dense or gas or config3" > $OUT/g3_dpp_tests.log 2>&1
echo done2
timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g3_sweep_base.jsonl 2> $OUT/g3_sweep_base.err
GNNREC_LIB=tools/bin/libgnnrec_exp64.so timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g3_sweep_exp64.jsonl 2> $OUT/g3_sweep_exp64.err
timeout -k 10 300 python tools/sweep_tiled.py 1117:49152:4096 > $OUT/g3_sweep_base2.jsonl 2> $OUT/g3_sweep_base2.err
echo done3
