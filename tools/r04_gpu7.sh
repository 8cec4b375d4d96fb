#!/bin/bash
# Round-4 GPU call 7: NGCF+GAS streaming transform A/B — shipped (12 waves, next tile's rows
# prefetched in registers) vs no prefetch at 12 and 16 waves per workgroup (build_variant libs);
# the transform alone on 2M rows, then config 3 (G100M NGCF+GAS) per library.
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/g7_transform.jsonl
: > $OUT/g7_config3.jsonl
for L in default tools/bin/libgnnrec_tf_np12.so tools/bin/libgnnrec_tf_np16.so; do
  if [ "$L" = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$L; fi
  echo "lib $L" >&2
  timeout -k 10 120 python -u tools/exp_transform.py >> $OUT/g7_transform.jsonl 2>> $OUT/g7_transform.err
  timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --steps 10 --no-ref-check \
      >> $OUT/g7_config3.jsonl 2>> $OUT/g7_config3.err
done
echo done
