set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wgb128; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_zb_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/kbench.py --c5 --ops wgrad_bf16 --iters 10 > $O/rel.txt 2>&1 || { tail -20 $O/rel.txt; exit 1; }
grep -v amdgpu.ids $O/rel.txt
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c5.json
