#!/bin/bash
# Round-4 GPU call 5: the whole -m gpu suite on the quad plan layout (ABI 9) and the v3
# transform; the transform's time decomposition (diagnostic builds: no MFMA / no GAS / no row
# loads; results wrong, timing only); the N=1 bench with the vendor comparator.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/ > $OUT/g5_gpu_tests.log 2>&1
for V in base texp1 texp2 texp4; do
  L=tools/bin/libgnnrec_$V.so; [ $V = base ] && L=gnn-recommendations_amd/lib/libgnnrec.so
  GNNREC_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/g5_tx_$V -o run -- python3 tools/bench_configs.py --configs 3 --steps 5 --no-ref-check \
      > $OUT/g5_tx_$V.jsonl 2> $OUT/g5_tx_$V.err
done
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/g5_bench.json 2> $OUT/g5_bench.err
echo done
