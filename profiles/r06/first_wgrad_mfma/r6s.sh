set -u
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_first_layer_gpu.py tests/test_train_gpu.py tests/test_probunet_gpu.py "tests/test_bf16_gpu.py::test_unet_autocast_bf16" "tests/test_bf16_gpu.py::test_c5_geometry_bf16_step_vs_oracle" "tests/test_bf16_gpu.py::test_c5_geometry_bf16_step_vs_oracle_batch16" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; cat $O/bitcmp.log
cd /tmp && export TMPDIR=/tmp
for lib in prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$lib -o b -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $GRAFT_REPO_ROOT/$O/prof_$lib.log 2>&1 || exit $?
  PMU_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof2_$lib -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof2_$lib.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv,glob
for lib in ['prev','rel']:
    for tag in ['prof','prof2']:
        f=glob.glob(f'gpurun_out/r6s/{tag}_{lib}/**/*kernel_stats.csv',recursive=True)[0]
        for r in csv.DictReader(open(f)):
            if 'first' in r['Name'] or 'rows_sum' in r['Name']:
                print(lib, tag, r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3), r['Name'][:80])
PY
