#!/bin/bash
# Round profile of the headline bench (run on the GPU box from the repo root):
#   bench.py with the CPU baseline, rocprofv3 kernel-trace stats, and the two PMC passes.
# usage: [BENCH_ARGS="--dim 128"] [NO_CPU=1] bash tools/profile_round.sh <tag>
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BA=${BENCH_ARGS:-}
CPU=""
[ -n "${NO_CPU:-}" ] && CPU="--no-cpu-baseline"
timeout -k 10 600 python bench.py $BA $CPU > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $BA --no-cpu-baseline --no-vendor --steps 10 > $OUT/kt_bench.json 2> $OUT/kt.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $BA --no-cpu-baseline --no-vendor --steps 3 --warmup 1 > $OUT/pmc_fetch_bench.json 2> $OUT/pmc_fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $BA --no-cpu-baseline --no-vendor --steps 3 --warmup 1 > $OUT/pmc_write_bench.json 2> $OUT/pmc_write.err
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- python3 bench.py $BA --no-cpu-baseline --no-vendor --steps 3 --warmup 1 > $OUT/pmc_l2_bench.json 2> $OUT/pmc_l2.err
K=${KERNEL:-tiled_hop_kernel}
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" -print -quit)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" -print -quit)
python tools/pmc_summarize.py "$F" "$W" $OUT/pmc_summary.json $K $OUT/pmc_fetch_bench.json
L=$(find $OUT/pmc_l2 -name "*counter_collection.csv" -print -quit)
python tools/pmc_l2.py "$L" > $OUT/l2_hit.txt
F2=$(find $OUT/kt -name "*kernel_stats.csv" -print -quit)
cp "$F2" $OUT/kernel_stats.csv
echo done
