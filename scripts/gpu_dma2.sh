# DMA bf16 kernels: parity tests, conv + convT kbench at c5 shapes, SQ counters of two conv shapes, c5 bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dma2; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -q -k "dma" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_dma.log 2>&1; rc=$?
tail -3 $O/tests_dma.log
if [ $rc -ne 0 ]; then grep -E "FAILED|assert|Error" $O/tests_dma.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/kbench.py --c5 --ops fwd_dma,dgrad_dma --iters 10 > $O/kbench_c5.txt 2>&1 || exit $?
grep TOTAL $O/kbench_c5.txt
timeout -k 10 300 python -u tools/kbench_convt.py --c5 --ops fwd_bf16,fwd_dma,dgrad_bf16,dgrad_dma,wgrad_bf16 --iters 10 > $O/kbench_convt_c5.txt 2>&1 || exit $?
grep TOTAL $O/kbench_convt_c5.txt
export TMPDIR=/tmp
for SH in "128,512,512" "1024,64,64"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $O/pmc_$SH -o p --output-format csv -- python tools/kbench.py --ops fwd_dma --only $SH --N 16 --iters 3 > $O/pmc_$SH.log 2>&1 || exit $?
done
python tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt | head -40
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-400 $O/bench_c5.json
