set -u
O=gpurun_out/r7c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_head_fuse_gpu.py tests/test_blocks_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head; exit $rc; }
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; cat $O/bitcmp.log
cd /tmp && export TMPDIR=/tmp
for v in prev rel; do
  L=$v; [ $v = rel ] && L=""
  PMU_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$v -o b -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || exit $?
  PMU_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof2_$v -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof2_$v.log 2>&1 || exit $?
  python3 - $GRAFT_REPO_ROOT/$O $v <<'PY'
import csv,glob,sys
for tag in ['prof','prof2']:
    f=glob.glob(sys.argv[1]+f'/{tag}_{sys.argv[2]}/**/*kernel_stats.csv',recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if 'head' in r['Name']: print(sys.argv[2], tag, r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3), r['Name'][:70])
PY
done
