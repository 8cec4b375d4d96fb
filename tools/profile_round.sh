#!/bin/bash
# One script for a round's GPU records (run on the GPU box from the repo root); every step
# under its own time limit, chained so the first failure ends the call.
#
#   bash tools/profile_round.sh <tag> [step ...]
#
# steps (default: tests smoke bench kt pmc):
#   tests   the whole -m gpu suite                        -> gpu_tests.log
#   smoke   __graft_entry__.smoke()                       -> smoke.log
#   bench   bench.py (CPU baseline + vendor comparators)  -> bench.json
#   kt      rocprofv3 --kernel-trace --stats of bench.py  -> kernel_stats.csv, kt_bench.json
#   pmc     FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes -> pmc_summary.json, l2_hit.txt
#   configs tools/bench_configs.py $CONFIGS (default "2 3 4 5 6 9") -> configs.jsonl
#   g1b     config 5 at full size (10M x 10M, 1B pairs), sampled-row oracle check -> config5_g1b.jsonl
#   c5kt    config 5 (5M x 5M) under the kernel tracer    -> c5_kernel_stats.csv
#   csr     tools/exp_csr_hop.py --powerlaw --g100m (config 2 + CSR paths) -> csr_hop.jsonl
#   c2kt    config 2's propagation under the kernel tracer -> c2_kernel_trace.csv
#   shards  tools/shard_compute.py (N-GPU compute side on one GPU) -> shard_compute.jsonl
#   hybrid  tools/exp_hybrid_hop.py (power-law hybrid hop estimate) -> hybrid.jsonl
# env: BENCH_ARGS (e.g. "--dim 128"), NO_CPU=1 (bench without the CPU baseline),
#      KERNEL (the PMC summary's kernel, default tiled_hop_kernel), TESTS (pytest selection)
set -euo pipefail
TAG=${1:?usage: profile_round.sh <tag> [step ...]}
shift
STEPS=${*:-tests smoke bench kt pmc}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BA=${BENCH_ARGS:-}
NOPROF="--no-cpu-baseline --no-vendor"
for step in $STEPS; do
  echo "[profile_round] $step" >&2
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
          ${TESTS:-tests/} > $OUT/gpu_tests.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
          > $OUT/smoke.log 2>&1 ;;
    bench)
      CPU=""
      [ -n "${NO_CPU:-}" ] && CPU="--no-cpu-baseline"
      timeout -k 10 600 python bench.py $BA $CPU > $OUT/bench.json 2> $OUT/bench.err ;;
    kt)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
          python3 bench.py $BA $NOPROF --steps 10 > $OUT/kt_bench.json 2> $OUT/kt.err
      cp "$(find $OUT/kt -name "*kernel_stats.csv" -print -quit)" $OUT/kernel_stats.csv ;;
    pmc)
      for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:l2"; do
        ctr=${pass%%:*}; name=${pass##*:}
        timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$name -o run -- \
            python3 bench.py $BA $NOPROF --steps 3 --warmup 1 > $OUT/pmc_${name}_bench.json \
            2> $OUT/pmc_$name.err
      done
      python tools/pmc_summarize.py "$(find $OUT/pmc_fetch -name "*counter_collection.csv" -print -quit)" \
          "$(find $OUT/pmc_write -name "*counter_collection.csv" -print -quit)" $OUT/pmc_summary.json \
          ${KERNEL:-tiled_hop_kernel} $OUT/pmc_fetch_bench.json
      python tools/pmc_table.py --l2 "$(find $OUT/pmc_l2 -name "*counter_collection.csv" -print -quit)" \
          > $OUT/l2_hit.txt ;;
    configs)
      timeout -k 10 900 python -u tools/bench_configs.py --configs ${CONFIGS:-2 3 4 5 6 9} \
          > $OUT/configs.jsonl 2> $OUT/configs.err ;;
    g1b)
      timeout -k 10 900 python -u tools/bench_configs.py --configs 5 --g1b --steps 5 \
          > $OUT/config5_g1b.jsonl 2> $OUT/config5_g1b.err ;;
    c5kt)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5kt -o run -- \
          python3 tools/bench_configs.py --configs 5 --c5-shape 5000000 5000000 250000000 --steps 3 \
          --warmup 1 --no-ref-check > $OUT/c5kt.jsonl 2> $OUT/c5kt.err
      cp "$(find $OUT/c5kt -name "*kernel_stats.csv" -print -quit)" $OUT/c5_kernel_stats.csv ;;
    csr)
      timeout -k 10 600 python -u tools/exp_csr_hop.py --tag $TAG --powerlaw --g100m \
          > $OUT/csr_hop.jsonl 2> $OUT/csr_hop.err ;;
    c2kt)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c2kt -o run -- \
          python3 tools/exp_csr_hop.py --tag $TAG --one ${C2_KNOBS:-0:2048:256} > $OUT/c2kt.jsonl 2> $OUT/c2kt.err
      cp "$(find $OUT/c2kt -name "*kernel_trace.csv" -print -quit)" $OUT/c2_kernel_trace.csv ;;
    shards)
      timeout -k 10 600 python -u tools/shard_compute.py > $OUT/shard_compute.jsonl 2> $OUT/shard_compute.err ;;
    hybrid)
      timeout -k 10 600 python -u tools/exp_hybrid_hop.py > $OUT/hybrid.jsonl 2> $OUT/hybrid.err ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo done
