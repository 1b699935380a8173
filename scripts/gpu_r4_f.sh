# Round-4 step F: (1) the tall 64-channel LDS-DMA conv shape (8 waves over 32 tile rows, one workgroup
# per CU; experiments build, PMU_DMA_TALL=1): parity tests, kbench and c5 bench A/B against the same
# library without it; (2) SQ counters of the F(4x4) input gradient on the K-short 256^2 c2 shapes.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4f; mkdir -p $O
cd $R
PMU_LIB=exp PMU_DMA_TALL=1 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_bf16_gpu.py tests/test_bnr_gpu.py -k "dma" > $O/tests_tall.log 2>&1 || { tail -30 $O/tests_tall.log; exit 1; }
tail -2 $O/tests_tall.log
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_bf16_gpu.py tests/test_bnr_gpu.py -k "dma" > $O/tests_rel.log 2>&1 || { tail -30 $O/tests_rel.log; exit 1; }
tail -1 $O/tests_rel.log
for T in 0 1; do
  PMU_LIB=exp PMU_DMA_TALL=$T timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab --iters 5 > $O/kbench_c5_tall$T.txt 2>&1 || exit $?
  grep TOTAL $O/kbench_c5_tall$T.txt
done
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_convT_gpu.py > $O/tests_convT.log 2>&1 || { tail -30 $O/tests_convT.log; exit 1; }
tail -1 $O/tests_convT.log
for T in 0 1; do
  PMU_LIB=exp PMU_DMA_TALL=$T timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_tall$T.json 2> $O/bench_c5_tall$T.err || exit $?
  cut -c 1-160 $O/bench_c5_tall$T.json
done
# the paired bf16 ConvT forward stores: release library vs the previous one (commit 29c9cac)
for L in prev rel; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$L.json 2> $O/bench_c5_$L.err || exit $?
  cut -c 1-160 $O/bench_c5_$L.json
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU GRBM_COUNT"
for S in 256,64,64 256,128,64 64,512,512; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1)); T=w4_$(echo $S | tr , _)_p$i
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/$T -o run -- python3 $R/tools/kbench.py --only $S --ops dgrad_w4 --iters 2 > $O/$T.log 2>&1 || exit $?
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*w4_$(echo $S | tr , _)_p*" -name "*counter_collection.csv") > $O/sq_w4_$(echo $S | tr , _).txt || exit $?
done
grep -A17 "wino4" $O/sq_w4_256_64_64.txt | head -20
