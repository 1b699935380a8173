# Round 4, step J: one-launch BatchNorm statistics with per-channel-block tickets — its tests, then
# (The one-launch BatchNorm-statistics kernels this A/B measured equal and were not kept)
# c5 / c2 bench A/B against the two-launch form (PMU_BN_STATS=0) on the same box.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepJ; mkdir -p $O
cd $R
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -q tests/test_bn_stats_gpu.py tests/test_pack_gpu.py tests/test_unet_gpu.py > $O/tests_new.log 2>&1 || { tail -30 $O/tests_new.log; exit 1; }
tail -2 $O/tests_new.log
for i in 1 2; do
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_fused_$i.json 2> $O/bench_c5.err || exit 1
PMU_BN_STATS=0 timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_two_$i.json 2> $O/bench_c5.err || exit 1
done
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c2_fused.json 2> $O/bench_c2.err || exit 1
PMU_BN_STATS=0 timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c2_two.json 2> $O/bench_c2.err || exit 1
for f in $O/bench_*.json; do echo "$(basename $f) $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'])")"; done
