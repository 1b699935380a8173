# Round-4 step H: fixed-order fp64 row sums (head and first-layer weight-gradient slabs) with 16 row
# phases x 4 accumulators per 1024-thread block.  Touched-kernel tests, then c5 / c2 bench A/B against
# PMU_LIB=prev (commit 8d32157).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4h; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_bnr_gpu.py tests/test_first_layer_gpu.py tests/test_unet_gpu.py tests/test_blocks_gpu.py \
  tests/test_probunet_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$L.json 2> $O/bench_c5_$L.err || exit $?
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_$L.json 2> $O/bench_c2_$L.err || exit $?
  cut -c 1-160 $O/bench_c5_$L.json $O/bench_c2_$L.json
done
