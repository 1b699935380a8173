# bf16-z storage: new kernel tests first, then the full GPU suite, the c5 bench (both z modes) and a
# c5 rocprof stats run into gpurun_out/zb.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/zb; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_zb_gpu.py -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests_zb.log 2>&1; rc=$?
tail -3 $O/tests_zb.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests_zb.log | head -30; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -x > $O/tests_gpu.log 2>&1; rc=$?
tail -3 $O/tests_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c5.json
PMU_BF16_Z=0 timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5_z32.json 2> $O/bench_c5_z32.err || exit $?
cut -c 1-200 $O/bench_c5_z32.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
echo done
