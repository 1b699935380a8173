set -u
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_first_layer_gpu.py tests/test_head_fuse_gpu.py tests/test_blocks_gpu.py tests/test_train_gpu.py tests/test_probunet_gpu.py "tests/test_bf16_gpu.py::test_c5_geometry_bf16_step_vs_oracle" "tests/test_bf16_gpu.py::test_c5_geometry_bf16_step_vs_oracle_batch16" "tests/test_bf16_gpu.py::test_unet_autocast_bf16" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; cat $O/bitcmp.log
cd /tmp && export TMPDIR=/tmp
for v in prev rel exphu4; do
  L=$v; H=""; [ $v = rel ] && L=""; [ $v = exphu4 ] && { L=exp; H=4; }
  PMU_LIB=$L PMU_HEAD_HU=$H timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$v -o b -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || exit $?
  PMU_LIB=$L PMU_HEAD_HU=$H timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof2_$v -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof2_$v.log 2>&1 || exit $?
  python3 - $GRAFT_REPO_ROOT/$O $v <<'PY'
import csv,glob,sys
for tag in ['prof','prof2']:
    f=glob.glob(sys.argv[1]+f'/{tag}_{sys.argv[2]}/**/*kernel_stats.csv',recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if 'head' in r['Name'] or 'first' in r['Name']: print(sys.argv[2], tag, r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3), r['Name'][:70])
PY
done
cd $GRAFT_REPO_ROOT
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/c5_$lib.json 2> $O/c5_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/c5_$lib.json'));print('c5 $lib', d['value'], d['ms_per_step'])"
done
