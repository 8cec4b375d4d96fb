#!/bin/bash
# Deferred layer-mean epilogue (hop 3: three base inputs per row): rows per half-wave batch.
# Run on the GPU box from the repo root after build_native.py + tools/build_variant.sh.
set -euo pipefail
OUT=gpurun_out/exp_epi3
mkdir -p $OUT
: > $OUT/epi3.jsonl  # variants: default = the in-tree build
VARIANTS=${VARIANTS:-default epi3_6 epi3_14 epi3_18}
for v in $VARIANTS; do
  if [ "$v" = default ]; then lib=gnn-recommendations_amd/lib/libgnnrec.so; else lib=${VARDIR:-tools/var_so}/$v.so; fi
  GNNREC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $OUT/b_$v.json 2> $OUT/b_$v.err
  python -c "import json,sys; d=json.load(open('$OUT/b_$v.json')); print(json.dumps({'batch3': '$v', 'ms_per_step': d['ms_per_step'], 'launch_ms': d['roofline']['launch_ms'], 'per_hop': d['roofline']['launch_ms_per_hop']}))" >> $OUT/epi3.jsonl
done
cat $OUT/epi3.jsonl
