#!/bin/bash
# Experiment builds: libgnnrec with extra -D flags on ONE kernel source, linked from the
# in-tree objects of the others (run after build_native.py). Load with GNNREC_LIB=<out>.
#   bash tools/build_variant.sh <out.so> <source.hip> -DNAME=VALUE ...
set -euo pipefail
OUT=$1; SRC=$2; shift 2
B=gnn-recommendations_amd/build
mkdir -p "$(dirname "$OUT")"
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt "$@" -c "gnn-recommendations_amd/csrc/$SRC" -o "$T/v.o"
OBJS=$(ls $B/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS "$T/v.o" -lpthread
rm -rf "$T"
echo "$OUT"
