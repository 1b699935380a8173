# Round 4, part B: the test fixed after the ABI split, c2 / c5 bench lines, MFMA counter calibration and
# the SQ counters of the DMA conv kernels.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4b; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wino4_gpu.py > $O/tests_wino4.log 2>&1 || { tail -20 $O/tests_wino4.log; exit 1; }
tail -1 $O/tests_wino4.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c2.json $O/bench_c5.json
bash scripts/gpu_mfma_calib.sh || exit $?
bash scripts/gpu_sq_dma.sh || exit $?
