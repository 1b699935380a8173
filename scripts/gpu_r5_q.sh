# Round 5: BN statistics in one launch (pmu_bn_{fwd,bwd}_stats, PMU_BN_FUSE) and the float4 Winograd
# split-K reduction.  Tests (release + debug), kernel-trace stats, c2 / c4 / c5 bench A/B
# (prev = the old reduction with the new BN kernels; cur with PMU_BN_FUSE=0/1).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5q; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bn_fuse_gpu.py tests/test_wino_gpu.py tests/test_wgrad4_gpu.py tests/test_bnr_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bn_fuse_gpu.py > $O/tests_debug.log 2>&1; rc=$?
tail -2 $O/tests_debug.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c2.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in "PMU_LIB=prev PMU_BN_FUSE=0" "PMU_LIB= PMU_BN_FUSE=0" "PMU_LIB= PMU_BN_FUSE=1"; do
    tag=$(echo $v | tr -d ' =_')
    env $v timeout -k 10 600 python bench.py --no-cpu-baseline --steps 20 > $O/bench_c2_${tag}_$i.json 2> $O/bench_c2_${tag}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c2_${tag}_$i.json'));print('c2 $v', d['value'], d['ms_per_step'])"
  done
done
for i in 1 2; do
  for v in "PMU_LIB=prev PMU_BN_FUSE=0" "PMU_LIB= PMU_BN_FUSE=1"; do
    tag=$(echo $v | tr -d ' =_')
    env $v timeout -k 10 600 python bench.py --workload probunet --no-cpu-baseline --steps 10 > $O/bench_c4_${tag}_$i.json 2> $O/bench_c4_${tag}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c4_${tag}_$i.json'));print('c4 $v', d['value'], d['ms_per_step'])"
    env $v timeout -k 10 600 python bench.py --workload c5 --no-eval --no-cpu-baseline --steps 10 > $O/bench_c5_${tag}_$i.json 2> $O/bench_c5_${tag}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c5_${tag}_$i.json'));print('c5 $v', d['value'], d['ms_per_step'])"
  done
done
echo r5q-done
