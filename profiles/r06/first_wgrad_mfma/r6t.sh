set -u
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_first_layer_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for v in rel exp8 rel exp8; do
  L=""; D=""; [ $v = exp8 ] && { L=exp; D=8; }
  PMU_LIB=$L PMU_FIRST_WG_DEPTH=$D timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$v -o b -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || exit $?
  python3 - $GRAFT_REPO_ROOT/$O/prof_$v $v <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'first' in r['Name']: print(sys.argv[2], r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3), r['Name'][:70])
PY
done
