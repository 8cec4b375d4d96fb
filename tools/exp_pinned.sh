#!/bin/bash
# Plan-shape A/B of the column-ordered hop on G100M d=64 (tools/sweep_tiled.py): panel plans
# (step barriers) vs pinned rows (panel 0) vs wave partitions (panel -1), for the shipped
# 8-wave kernel and 12 / 16-wave variant builds (tools/build_variant.sh into tools/bin/).
#   bash tools/exp_pinned.sh <out.jsonl>
set -uo pipefail
OUT=$1
: > "$OUT"
run() {   # name waves lib shapes...
  local name=$1 waves=$2 lib=$3; shift 3
  GNNREC_TILED_WAVES=$waves GNNREC_LIB=$lib timeout -k 10 300 python -u tools/sweep_tiled.py "$@" 2>&1 \
    | grep "^{" | sed "s/^{/{\"variant\": \"$name\", /" >> "$OUT" || { echo "variant $name failed"; exit 1; }
}
run w8 8 gnn-recommendations_amd/lib/libgnnrec.so 1117:49152:4096 1117:0:4096 1117:-1:4096 1117:-1:2048 977:-1:4096
run w12 12 tools/bin/w12.so 1117:0:4096 1117:-1:4096
run w16p2g1 16 tools/bin/w16p2g1.so 1117:0:4096 1117:-1:4096
cat "$OUT"
