#!/bin/bash
# XCD-group start stagger for the column-ordered hop (A/B): each setting in its own bench
# process (the library reads GNNREC_TILED_STAGGER_NS / _EPI once). Settings "ns:epi_mask",
# epi mask 16 = hop 3 (ACC_X) only, -1 = every hop. The hook (thread 0 of each workgroup
# sleeping (blockIdx % 8) x ns before its first pass) was removed after the A/B
# (profiles/r06/tiled_xcd_stagger.jsonl, no gain); re-add it to tiled.hip to re-run.
#   bash tools/exp_stagger.sh [setting ...]
set -euo pipefail
OUT=gpurun_out/stagger
mkdir -p $OUT
for st in ${*:-0:16 4000:16 8000:16 16000:16 4000:-1 0:16}; do
  ns=${st%%:*}; mask=${st##*:}
  GNNREC_TILED_STAGGER_NS=$ns GNNREC_TILED_STAGGER_EPI=$mask timeout -k 10 300 \
      python bench.py --no-cpu-baseline --no-vendor --steps 30 > $OUT/b_${ns}_${mask}.json 2> $OUT/b_${ns}_${mask}.err
  python - "$ns" "$mask" "$OUT/b_${ns}_${mask}.json" >> $OUT/stagger.jsonl <<'EOF'
import json, sys
r = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(json.dumps({"stagger_ns": int(sys.argv[1]), "epi_mask": int(sys.argv[2]),
                  "ms_per_step": r["ms_per_step"], "launch_ms_per_hop": r["roofline"]["launch_ms_per_hop"]}))
EOF
  tail -1 $OUT/stagger.jsonl
done
