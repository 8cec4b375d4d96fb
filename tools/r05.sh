#!/bin/bash
# Round-5 GPU calls (one file for the round; each call is a case). Run from the repo root on
# the GPU box:  bash tools/r05.sh <call>
set -euo pipefail
OUT=gpurun_out/r05
mkdir -p $OUT
export TMPDIR=/tmp
C5="--configs 5 --c5-shape 5000000 5000000 250000000"
case ${1:?call} in
  c1)
    # the whole -m gpu suite after the round's first changes, the headline bench with the
    # rocSPARSE comparator, config 5 at 5M x 5M with the sampled-row oracle check, and the
    # GAT kernels' L2 hit/miss and fabric bytes at that size
    timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ \
        > $OUT/c1_gpu_tests.log 2>&1
    timeout -k 10 600 python bench.py > $OUT/c1_bench.json 2> $OUT/c1_bench.err
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c1_config5_g250m.jsonl \
        2> $OUT/c1_config5_g250m.err
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c1_c5kt -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c1_c5kt.jsonl 2> $OUT/c1_c5kt.err
    timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/c1_c5l2 -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c1_c5l2.jsonl 2> $OUT/c1_c5l2.err
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c1_c5fetch -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c1_c5fetch.jsonl 2> $OUT/c1_c5fetch.err
    ;;
  c2)
    # scores-from-rows GAT kernels (ABI 10): their tests and the GAT model / golden tests,
    # config 5 at 5M x 5M (checked) + its kernel trace, then G1B with the sampled-row check
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_models_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_offsets_gpu.py tests/test_tiled_plan_gpu.py > $OUT/c2_gat_tests.log 2>&1
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c2_config5_g250m.jsonl \
        2> $OUT/c2_config5_g250m.err
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_c5kt -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c2_c5kt.jsonl 2> $OUT/c2_c5kt.err
    timeout -k 10 900 python -u tools/bench_configs.py --configs 5 --g1b --steps 5 \
        > $OUT/c2_config5_g1b.jsonl 2> $OUT/c2_config5_g1b.err
    ;;
  c3)
    # A/B of the ATT GAT kernel builds (tools/var/gat_*.so, built on the CPU with
    # tools/build_variant.sh) and the score-table kernels, config 5 at 5M x 5M, same box
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_gat_train_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py > $OUT/c3_gat_tests.log 2>&1 || true
    : > $OUT/c3_gat_variants.jsonl
    GNNREC_GAT_SCORES_FROM_ROWS=0 timeout -k 10 300 python -u tools/exp_gat_variants.py --tag tables \
        >> $OUT/c3_gat_variants.jsonl 2> $OUT/c3.err
    for v in ch16w4 ch8w6 ch8w5 ch16w4_nolds ch16w4; do
      GNNREC_LIB=tools/var/gat_$v.so timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v \
          >> $OUT/c3_gat_variants.jsonl 2>> $OUT/c3.err
    done
    GNNREC_GAT_SEGMENT_ORDER=row GNNREC_GAT_XCD_ORDER=0 GNNREC_LIB=tools/var/gat_ch16w4.so \
        timeout -k 10 300 python -u tools/exp_gat_variants.py --tag ch16w4_roworder >> $OUT/c3_gat_variants.jsonl 2>> $OUT/c3.err
    GNNREC_GAT_XCD_ORDER=0 GNNREC_LIB=tools/var/gat_ch16w4.so \
        timeout -k 10 300 python -u tools/exp_gat_variants.py --tag ch16w4_colorder_noxcd >> $OUT/c3_gat_variants.jsonl 2>> $OUT/c3.err
    ;;
  c4)
    # the chosen ATT build: G1B kernel trace (checked run before it), and the GAT kernels'
    # L2 hit / miss at 5M x 5M
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_g1bkt -o run -- \
        python3 tools/bench_configs.py --configs 5 --g1b --steps 3 --warmup 1 --no-ref-check \
        > $OUT/c4_g1bkt.jsonl 2> $OUT/c4_g1bkt.err
    timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/c4_c5l2 -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c4_c5l2.jsonl 2> $OUT/c4_c5l2.err
    ;;
  c5)
    # heavy-row segment plans, same box: equal-length by first column (default) vs panel-cut
    : > $OUT/c5_gat_panels.jsonl
    timeout -k 10 300 python -u tools/exp_gat_variants.py --tag column >> $OUT/c5_gat_panels.jsonl 2> $OUT/c5.err
    for pp in "8192 64" "16384 64" "4096 64" "8192 256" "32768 64"; do
      set -- $pp
      GNNREC_GAT_SEGMENT_ORDER=panel GNNREC_GAT_PANEL=$1 GNNREC_GAT_PANEL_MIN_EDGES=$2 \
          timeout -k 10 300 python -u tools/exp_gat_variants.py --tag panel_$1_$2 \
          >> $OUT/c5_gat_panels.jsonl 2>> $OUT/c5.err
    done
    timeout -k 10 300 python -u tools/exp_gat_variants.py --tag column >> $OUT/c5_gat_panels.jsonl 2>> $OUT/c5.err
    GNNREC_LIB=tools/var/gat_ch16w4_nolds.so timeout -k 10 300 python -u tools/exp_gat_variants.py \
        --tag nolds_fixed >> $OUT/c5_gat_panels.jsonl 2>> $OUT/c5.err
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5_c5kt -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c5_c5kt.jsonl 2> $OUT/c5_c5kt.err
    ;;
  c6)
    # the shared-row (last GAT layer) kernel: next block's rows in flight (GAT_SHARED_PIPE)
    # at 3 or 4 waves per SIMD, same box, 5M x 5M; then correctness of the chosen default
    : > $OUT/c6_gat_pipe.jsonl
    for v in default pipe3 pipe4 w3 default; do
      L=tools/var/gat_$v.so; [ $v = default ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v \
          >> $OUT/c6_gat_pipe.jsonl 2>> $OUT/c6.err
    done
    GNNREC_LIB=tools/var/gat_pipe3.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/c6_pipe3kt -o run -- python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check \
        > $OUT/c6_pipe3kt.jsonl 2> $OUT/c6_pipe3kt.err
    ;;
  c7)
    # the head-major kernel with the next chunk in flight (GAT_MAIN_PIPE, 8 + 8 neighbours)
    : > $OUT/c7_gat_mpipe.jsonl
    for v in default mpipe8 default mpipe8; do
      L=tools/var/gat_$v.so; [ $v = default ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v \
          >> $OUT/c7_gat_mpipe.jsonl 2>> $OUT/c7.err
    done
    ;;
  c8)
    # cold-tail rows gathered non-temporal (GAT_HOT_COLS: ids below it are the hot rows of the
    # degree-ordered Zipf graph), same box, 5M x 5M
    : > $OUT/c8_gat_hot.jsonl
    for v in default hot16384 hot65536 hot262144 default; do
      L=tools/var/gat_$v.so; [ $v = default ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v \
          >> $OUT/c8_gat_hot.jsonl 2>> $OUT/c8.err
    done
    ;;
  c9)
    # heavy-segment plans at full G1B (its heaviest rows are 3x those of 5M x 5M), one process
    timeout -k 10 900 python -u tools/exp_gat_variants.py --tag g1b --shape 10000000 10000000 1000000000 \
        --reps 5 --plans column panel:8192:256 panel:16384:256 panel:8192:64 panel:32768:512 column \
        > $OUT/c9_g1b_plans.jsonl 2> $OUT/c9.err
    ;;
  c10)
    # stall decomposition of the shared-row kernel (2M x 2M slice), scores from rows vs tables
    S="python3 tools/exp_gat_variants.py --tag st --shape 2000000 2000000 50000000 --reps 3"
    bash tools/pmc_stalls_kernel.sh $OUT/c10_att gat_shared_kernel -- $S
    GNNREC_GAT_SCORES_FROM_ROWS=0 bash tools/pmc_stalls_kernel.sh $OUT/c10_tab gat_shared_kernel -- $S
    ;;
  c11)
    # the final GAT default (panel-cut heavy rows): GAT GPU tests, config 5 at 5M x 5M and at
    # G1B, both with the sampled-row check
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_gat_train_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py tests/test_fullsize_models_gpu.py > $OUT/c11_gat_tests.log 2>&1
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c11_config5_g250m.jsonl \
        2> $OUT/c11_config5_g250m.err
    timeout -k 10 800 python -u tools/bench_configs.py --configs 5 --g1b --steps 5 \
        > $OUT/c11_config5_g1b.jsonl 2> $OUT/c11_config5_g1b.err
    ;;
  c12)
    # config 5's heavy rows alone: CSR SpMM vs the column-ordered tiled hop vs the GAT heavy
    # partials on the same rows (is an LDS-resident schedule worth building for them?)
    for band in ${BANDS:-2048:65536 2048:0 0:2048}; do
      timeout -k 10 300 python -u tools/exp_heavy_tiled.py --lo ${band%:*} --hi ${band#*:} \
          >> $OUT/c12_heavy_tiled.jsonl 2>> $OUT/c12_heavy_tiled.err
    done
    ;;
  c13)
    # rows_gemm with the B operand as LDS fragments (ds_read_b128 per 4 MFMA steps): its tests,
    # then the GEMMs alone and config 5 at 5M x 5M, same box, against the round's base build
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py -k "rows_gemm" tests/test_gat_att_gpu.py > $OUT/c13_tests.log 2>&1
    : > $OUT/c13_rows_gemm.jsonl; : > $OUT/c13_gat.jsonl
    for v in base new base new; do
      L=tools/ab/base_r05.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_rows_gemm.py --tag $v >> $OUT/c13_rows_gemm.jsonl 2>> $OUT/c13.err
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c13_gat.jsonl 2>> $OUT/c13.err
    done
    ;;
  c14)
    # rows_gemm final (fragments for K >= 128 only): tests + timing; the NGCF transform with
    # its waves started apart (GNNREC_TRANSFORM_STAGGER), same box
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_gat_att_gpu.py > $OUT/c14_tests.log 2>&1
    timeout -k 10 120 python -u tools/exp_rows_gemm.py --tag final > $OUT/c14_rows_gemm.jsonl 2> $OUT/c14.err
    : > $OUT/c14_transform.jsonl
    for v in default 8 20 40 100 default 20 40; do
      L=tools/ab/tr_stagger$v.so; [ $v = default ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_transform.py | sed "s/^{/{\"variant\": \"$v\", /" \
          >> $OUT/c14_transform.jsonl 2>> $OUT/c14.err
    done
    ;;
  c15)
    # unconditional prefetch loads in the streaming MFMA kernels (transform64, rows_gemm): the
    # compiler had waited for the next tile's rows right after issuing them. Tests, then same-box
    # A/B against the previous source (tools/ab/head_r05.so): kernels alone, config 3 traced
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_gat_att_gpu.py tests/test_models_gpu.py \
        tests/test_fullsize_models_gpu.py > $OUT/c15_tests.log 2>&1
    : > $OUT/c15_transform.jsonl; : > $OUT/c15_rows_gemm.jsonl; : > $OUT/c15_config3.jsonl
    for v in head new head new; do
      L=tools/ab/head_r05.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_transform.py | sed "s/^{/{\"variant\": \"$v\", /" \
          >> $OUT/c15_transform.jsonl 2>> $OUT/c15.err
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_rows_gemm.py --tag $v >> $OUT/c15_rows_gemm.jsonl 2>> $OUT/c15.err
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --steps 10 --no-ref-check \
          | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/c15_config3.jsonl 2>> $OUT/c15.err
    done
    for v in head new; do
      L=tools/ab/head_r05.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c15_c3kt_$v -o run -- \
          python3 tools/bench_configs.py --configs 3 --steps 5 --warmup 1 --no-ref-check > $OUT/c15_c3kt_$v.jsonl 2>> $OUT/c15.err
    done
    ;;
  c16)
    # the kept form (unconditional prefetch for the NGCF transform and rows_gemm K >= 128 only):
    # tests, then the kernels alone against the previous source
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_fullsize_models_gpu.py \
        tests/test_gat_att_gpu.py > $OUT/c16_tests.log 2>&1
    : > $OUT/c16_transform.jsonl; : > $OUT/c16_rows_gemm.jsonl
    for v in head new head new; do
      L=tools/ab/head_r05.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_transform.py | sed "s/^{/{\"variant\": \"$v\", /" \
          >> $OUT/c16_transform.jsonl 2>> $OUT/c16.err
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_rows_gemm.py --tag $v >> $OUT/c16_rows_gemm.jsonl 2>> $OUT/c16.err
    done
    ;;
  c17)
    # GAT softmax normalisation by one reciprocal per head (gat_norm): GAT tests, then config 5
    # at 5M x 5M against the previous build, same box, and the checked run
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_gat_train_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py tests/test_fullsize_models_gpu.py > $OUT/c17_tests.log 2>&1
    : > $OUT/c17_gat.jsonl
    for v in base new base new; do
      L=tools/ab/pre_norm.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c17_gat.jsonl 2>> $OUT/c17.err
    done
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c17_config5_g250m.jsonl \
        2> $OUT/c17_config5_g250m.err
    ;;
  c18)
    # shared-row GAT kernel: 16 column indices per load serve two 8-neighbour blocks; GAT
    # tests, then config 5 at 5M x 5M against the previous build, same box
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_real_shapes_gpu.py tests/test_models_gpu.py \
        > $OUT/c18_tests.log 2>&1
    : > $OUT/c18_gat.jsonl
    for v in base new base new; do
      L=tools/ab/pre_shcol.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c18_gat.jsonl 2>> $OUT/c18.err
    done
    ;;
  c19)
    # final-tree GAT evidence: G1B kernel trace (checked run is final2), and the GAT kernels'
    # L2 hit / miss at 5M x 5M
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c19_g1bkt -o run -- \
        python3 tools/bench_configs.py --configs 5 --g1b --steps 3 --warmup 1 --no-ref-check \
        > $OUT/c19_g1bkt.jsonl 2> $OUT/c19_g1bkt.err
    timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/c19_c5l2 -o run -- \
        python3 tools/bench_configs.py $C5 --steps 3 --warmup 1 --no-ref-check > $OUT/c19_c5l2.jsonl 2> $OUT/c19_c5l2.err
    ;;
  c20)
    # cold-row gathers non-temporal when a whole wave's neighbours are cold (wave-uniform, one
    # load instruction), hot = degree rank < H on either side of the 5M x 5M graph; H = 1 (almost
    # all nt) and H = inf (branches only) bracket it. Same box, config 5 at 5M x 5M
    : > $OUT/c20_gat_hot.jsonl
    for v in default inf 1 4096 16384 65536 default 16384; do
      L=tools/ab/gat_hotu$v.so; [ $v = default ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag hot_$v \
          >> $OUT/c20_gat_hot.jsonl 2>> $OUT/c20.err
    done
    ;;
  c21)
    # GAT column indices broadcast by DPP row_newbcast instead of __shfl (ds_bpermute): GAT
    # tests, then config 5 at 5M x 5M against the previous build, same box
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_gat_train_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py > $OUT/c21_tests.log 2>&1
    : > $OUT/c21_gat.jsonl
    for v in base new base new; do
      L=tools/ab/pre_dpp.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c21_gat.jsonl 2>> $OUT/c21.err
    done
    ;;
  c22)
    # GAT gathers: single-instruction row addressing (row_at) everywhere, DPP index broadcast in
    # the head-major kernels only; tests, then config 5 at 5M x 5M against the build before
    # c21, same box
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_gat_train_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py tests/test_fullsize_models_gpu.py > $OUT/c22_tests.log 2>&1
    : > $OUT/c22_gat.jsonl
    for v in base new base new; do
      L=tools/ab/pre_dpp.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c22_gat.jsonl 2>> $OUT/c22.err
    done
    ;;
  c23)
    # shared-row GAT kernel: block max by DPP instead of __shfl_xor; GAT tests, then config 5
    # at 5M x 5M against the previous build, same box
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gat_att_gpu.py tests/test_real_shapes_gpu.py tests/test_models_gpu.py \
        > $OUT/c23_tests.log 2>&1
    : > $OUT/c23_gat.jsonl
    for v in base new base new; do
      L=tools/ab/pre_dppmax.so; [ $v = new ] && L=gnn-recommendations_amd/lib/libgnnrec.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c23_gat.jsonl 2>> $OUT/c23.err
    done
    ;;
  c24)
    # the final GAT build at full size: config 5 at 5M x 5M and at G1B, both checked
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c24_config5_g250m.jsonl \
        2> $OUT/c24_config5_g250m.err
    timeout -k 10 900 python -u tools/bench_configs.py --configs 5 --g1b --steps 5 \
        > $OUT/c24_config5_g1b.jsonl 2> $OUT/c24_config5_g1b.err
    ;;
  c32)
    # config 5 records with the roofline and request-model fields (5M x 5M and G1B, checked)
    timeout -k 10 600 python -u tools/bench_configs.py $C5 --steps 5 > $OUT/c32_config5_g250m.jsonl \
        2> $OUT/c32_config5_g250m.err
    timeout -k 10 900 python -u tools/bench_configs.py --configs 5 --g1b --steps 5 \
        > $OUT/c32_config5_g1b.jsonl 2> $OUT/c32_config5_g1b.err
    ;;
  c33)
    # configs 2-4 records with the roofline field (SURVEY 8(d) bytes, as the headline's)
    timeout -k 10 900 python -u tools/bench_configs.py --configs 2 3 4 --steps 10 \
        > $OUT/c33_configs_2_3_4.jsonl 2> $OUT/c33_configs_2_3_4.err
    ;;
  c34)
    # config 2 (ML-1M LightGCN) kernel trace: GPU time per forward against the 0.256 ms wall
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c34_kt -o run -- \
        python3 tools/bench_configs.py --configs 2 --steps 10 > $OUT/c34_config2.jsonl 2> $OUT/c34.err
    ;;
  c35)
    # CSR hop: indices one step ahead (vec kernel), 4 LDS steps ahead (heavy-row consumer).
    # The CSR / heavy-row / long-row GPU tests on the new build, then the same-box A/B
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_long_rows_gpu.py tests/test_offsets_gpu.py \
        tests/test_real_shapes_gpu.py > $OUT/c35_tests.log 2>&1
    for lib in tools/ab/base.so default tools/ab/nopipe.so tools/ab/ahead8.so default tools/ab/base.so; do
      if [ $lib = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$lib; fi
      timeout -k 10 300 python -u tools/exp_csr_hop.py --tag c35 --g100m \
          >> $OUT/c35_csr_hop.jsonl 2>> $OUT/c35.err
    done
    ;;
  c36)
    # the kept form (4 LDS steps ahead for the F = 1 heavy instances only, no index prefetch):
    # CSR / heavy / long-row GPU tests, then alternating same-box timings against round 4's
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_long_rows_gpu.py tests/test_offsets_gpu.py \
        tests/test_real_shapes_gpu.py tests/test_models_gpu.py > $OUT/c36_tests.log 2>&1
    for lib in tools/ab/base.so default tools/ab/base.so default; do
      if [ $lib = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$lib; fi
      timeout -k 10 300 python -u tools/exp_csr_hop.py --tag c36 >> $OUT/c36_csr_hop.jsonl 2>> $OUT/c36.err
    done
    ;;
  c37)
    # heavy-row consumer variants (B: unclamped read-ahead + a scheduling barrier per step so
    # each LDS fetch stays 4 steps ahead; C: 72 KB buffers, 284 neighbours per round at
    # d = 64; D: both): the CSR / heavy / long-row tests on D, then alternating timings
    GNNREC_LIB=tools/ab/D.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
        --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_long_rows_gpu.py \
        tests/test_offsets_gpu.py tests/test_real_shapes_gpu.py > $OUT/c37_tests.log 2>&1
    for lib in default tools/ab/B.so tools/ab/C.so tools/ab/D.so default tools/ab/B.so tools/ab/C.so tools/ab/D.so; do
      if [ $lib = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$lib; fi
      timeout -k 10 300 python -u tools/exp_csr_hop.py --tag c37 >> $OUT/c37_csr_hop.jsonl 2>> $OUT/c37.err
    done
    ;;
  c38)
    # the heavy-row change on the power-law 2M x 2M LightGCN (d = 64 and 128) and config 2,
    # against round 4's spmm.hip (tools/ab/r4.so), alternating
    for lib in tools/ab/r4.so default tools/ab/r4.so default; do
      if [ $lib = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$lib; fi
      timeout -k 10 300 python -u tools/exp_csr_hop.py --tag c38 --powerlaw >> $OUT/c38_csr_hop.jsonl 2>> $OUT/c38.err
    done
    ;;
  c39)
    # the new consumer for the d = 32 / 64 instances only (d = 128 and runtime d back to round
    # 4's form): CSR / heavy / long-row tests, then alternating timings against round 4
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_kernels_gpu.py tests/test_long_rows_gpu.py tests/test_offsets_gpu.py \
        tests/test_real_shapes_gpu.py tests/test_models_gpu.py > $OUT/c39_tests.log 2>&1
    for lib in tools/ab/r4.so default tools/ab/r4.so default; do
      if [ $lib = default ]; then unset GNNREC_LIB; else export GNNREC_LIB=$lib; fi
      timeout -k 10 300 python -u tools/exp_csr_hop.py --tag c39 --powerlaw >> $OUT/c39_csr_hop.jsonl 2>> $OUT/c39.err
    done
    ;;
  c25)
    # head-major GAT kernels with the chunk's scores pinned before its first block (all 16
    # gathers issued together instead of 8 + 8 behind the first block's work), same box
    GNNREC_LIB=tools/ab/gat_pin.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
        --timeout-method thread -m gpu tests/test_gat_att_gpu.py tests/test_real_shapes_gpu.py \
        tests/test_models_gpu.py > $OUT/c25_tests.log 2>&1
    : > $OUT/c25_gat.jsonl
    for v in base pin base pin; do
      L=gnn-recommendations_amd/lib/libgnnrec.so; [ $v = pin ] && L=tools/ab/gat_pin.so
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/exp_gat_variants.py --tag $v >> $OUT/c25_gat.jsonl 2>> $OUT/c25.err
    done
    ;;
  c26)
    # where the BPR training steps (configs 6 and 9) spend their time: kernel trace
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c26_trainkt -o run -- \
        python3 tools/bench_configs.py --configs 6 9 --steps 5 --warmup 2 > $OUT/c26_trainkt.jsonl 2> $OUT/c26_trainkt.err
    ;;
  c27)
    # heavy-row threshold / segment length at G1B, one process, same graph
    timeout -k 10 1000 python -u tools/exp_gat_variants.py --tag g1b --shape 10000000 10000000 1000000000 \
        --reps 5 --splits 2048:1024 1024:512 1024:1024 4096:1024 4096:2048 2048:512 2048:2048 2048:1024 \
        > $OUT/c27_g1b_splits.jsonl 2> $OUT/c27.err
    ;;
  c28)
    # NGCF + GAS transform software-pipelined per wave (GNNREC_TRANSFORM_PIPE=1, 8 waves per
    # workgroup): its tests, then the transform alone and config 3 against the shipped build
    GNNREC_LIB=tools/ab/tr_pipe8.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
        --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "ngcf or transform or gas" \
        > $OUT/c28_tests.log 2>&1
    GNNREC_LIB=tools/ab/tr_pipe8.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
        --timeout-method thread -m gpu tests/test_fullsize_models_gpu.py -k config3 >> $OUT/c28_tests.log 2>&1
    : > $OUT/c28_transform.jsonl; : > $OUT/c28_config3.jsonl
    for v in base pipe base pipe; do
      L=gnn-recommendations_amd/lib/libgnnrec.so; [ $v = pipe ] && L=tools/ab/tr_pipe8.so
      GNNREC_LIB=$L timeout -k 10 120 python -u tools/exp_transform.py | sed "s/^{/{\"variant\": \"$v\", /" \
          >> $OUT/c28_transform.jsonl 2>> $OUT/c28.err
      GNNREC_LIB=$L timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --steps 10 --no-ref-check \
          | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/c28_config3.jsonl 2>> $OUT/c28.err
    done
    GNNREC_LIB=tools/ab/tr_pipe8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/c28_c3kt_pipe -o run -- python3 tools/bench_configs.py --configs 3 --steps 5 --warmup 1 \
        --no-ref-check > $OUT/c28_c3kt_pipe.jsonl 2>> $OUT/c28.err
    ;;
  c30)
    # device planner with 16-bit run lengths in LDS (7 workgroups per CU: one round of blocks):
    # the planner tests (device == host plan, bit for bit), the tiled hop tests, then the bench
    # (operand prep phases) and a planner kernel trace
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_tiled_plan_gpu.py tests/test_long_rows_gpu.py tests/test_kernels_gpu.py \
        tests/test_offsets_gpu.py > $OUT/c30_tests.log 2>&1
    timeout -k 10 600 python bench.py --no-cpu-baseline --no-vendor > $OUT/c30_bench.json 2> $OUT/c30_bench.err
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c30_kt -o run -- \
        python3 bench.py --no-cpu-baseline --no-vendor --steps 5 > $OUT/c30_kt.json 2> $OUT/c30_kt.err
    ;;
  c31)
    # the N = 2 bench path on the final tree, rehearsed on one GPU with gloo (host-staged
    # exchange, not RCCL): layouts, exchange candidates, the default self-check and its labels
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo \
        --steps 3 --warmup 1 --no-cpu-baseline --no-vendor > $OUT/c31_n2_gloo.json 2> $OUT/c31_n2_gloo.err
    ;;
  *) echo "unknown call $1" >&2; exit 2 ;;
esac
echo done
