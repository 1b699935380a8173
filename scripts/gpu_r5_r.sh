# Round 5: the c4 eval's Dice counts of all 16 samples in one launch (pmu_dice_counts_many).  Dice /
# ProbUNet tests, c4 kernel-trace stats, c4 bench x3.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5r; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_data_gpu.py tests/test_probunet_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o bench -- python3 $R/bench.py --workload probunet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c4.log 2>&1 || exit $?
cd $R
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --workload probunet --no-cpu-baseline --steps 20 > $O/bench_c4_$i.json 2> $O/bench_c4_$i.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c4_$i.json'));print('c4', d['value'], d['ms_per_step'])"
done
echo r5r-done
