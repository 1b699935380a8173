# Round 5: the pooled layer's da left unstored (PoolSumDa: stats-only max-pool backward + fused
# max-pool/BN-backward dz pass).  New tests (release, then the bounds-checked debug build), the dx-bf16
# tests, then c5 bench A/B (PMU_POOL_FUSE=0/1).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_pool_fuse_gpu.py > $O/fuse_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error" $O/fuse_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_pool_fuse_gpu.py > $O/fuse_tests_debug.log 2>&1; rc=$?
tail -2 $O/fuse_tests_debug.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_dxb_gpu.py tests/test_bf16_gpu.py -k "unet or c5 or maxpool" > $O/model_tests.log 2>&1; rc=$?
tail -2 $O/model_tests.log
[ $rc -ne 0 ] && exit $rc
for f in 0 1 0 1; do
  PMU_POOL_FUSE=$f timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_fuse$f.json 2> $O/bench_c5_fuse$f.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_fuse$f.json'));print('fuse=$f', d['value'], d['ms_per_step'])"
done
echo r5h-done
