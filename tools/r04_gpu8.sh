#!/bin/bash
# Round-4 GPU call 8: (1) the transform A/B again with the GAS permutation drawn from the
# seeded generator (the first run used the default generator) plus an in-process repeat and a
# torch fp32 reference diff per library; (2) config 5 at 5M x 5M (250M pairs) under the
# kernel tracer — the step before a traced G1B run (profiles/r03/g1b_box_loss_record.md).
set -euo pipefail
OUT=gpurun_out/r04
mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/g8_transform.jsonl
for L in default tools/bin/libgnnrec_tf_np12.so tools/bin/libgnnrec_tf_np16.so; do
  if [ "$L" = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$L; fi
  timeout -k 10 180 python -u tools/exp_transform.py >> $OUT/g8_transform.jsonl 2>> $OUT/g8_transform.err
done
unset GNNREC_LIB
timeout -k 10 300 python -u tools/exp_hop_context.py > $OUT/g8_hop_context.jsonl 2> $OUT/g8_hop_context.err
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g8_c5_g250m -o run -- \
    python3 -u tools/bench_configs.py --configs 5 --c5-shape 5000000 5000000 250000000 \
    --steps 5 --warmup 1 --no-ref-check > $OUT/g8_c5_g250m_kt.jsonl 2> $OUT/g8_c5_g250m_kt.err
echo done
