#!/bin/bash
# A/B of libgnnrec variants (tools/build_variant.sh) on the G100M d=64 hop: one
# tools/sweep_tiled.py run per variant library (GNNREC_LIB), one JSON line each, tagged.
#   bash tools/sweep_variants.sh <out.jsonl> <shape> [--fold N] <name=lib.so> ...
set -uo pipefail
OUT=$1; SHAPE=$2; shift 2
EXTRA=""
if [ "${1:-}" = "--fold" ]; then EXTRA="--fold $2"; shift 2; fi
: > "$OUT"
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  # name suffix "_explicit": the same library with explicit-value plans
  case "$name" in *_explicit) export TILED_FACTOR=0 ;; *) unset TILED_FACTOR ;; esac
  GNNREC_LIB=$lib timeout -k 10 200 python -u tools/sweep_tiled.py $EXTRA $SHAPE 2>&1 \
    | grep "^{" | sed "s/^{/{\"variant\": \"$name\", /" >> "$OUT" || { echo "variant $name failed"; exit 1; }
done
cat "$OUT"
