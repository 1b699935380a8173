set -u
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_probunet_gpu.py -k "concurrent or c4_geometry" tests/test_dp_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for f in 0 1; do
  PMU_PROB_STREAMS=$f timeout -k 10 300 python bench.py --workload probunet --no-cpu-baseline > $O/c4_s$f.json 2> $O/c4_s$f.err || exit $?
  python -c "import json;d=json.load(open('$O/c4_s$f.json'));print('c4 streams=$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline_next']['kernel'])"
done
timeout -k 10 900 python -u tools/dice_gap_seeds.py --seeds 0,1,2,3,4,5,6,7 --out $O/dice_gap_seeds.json > $O/dice_gap_seeds.log 2>&1; echo dice rc=$?
