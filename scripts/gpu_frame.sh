set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/frame; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_frame_stream_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python tools/kbench_frame.py --c5 > $O/c5.txt 2>&1 || { tail -20 $O/c5.txt; exit 1; }
grep -v amdgpu.ids $O/c5.txt
timeout -k 10 180 python tools/kbench_frame.py > $O/c2.txt 2>&1 || { tail -20 $O/c2.txt; exit 1; }
grep -v amdgpu.ids $O/c2.txt
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
  cut -c 1-200 $O/bench_c5.json
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
  cut -c 1-200 $O/bench_c2.json
fi
