# F(4x4) Winograd: parity tests, kernel A/B vs F(2x2) on the c2 shapes, c2 bench A/B
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/w4; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${TESTS:-tests/test_wino4_gpu.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/kbench.py --ops ${OPS:-fwd_wr,fwd_w4,dgrad_wr,dgrad_w4} --iters 10 > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
if [ -n "${BENCH:-}" ]; then
  for S in PMU_WINO4=0 PMU_WINO4=1; do
    env $S timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --steps 10 > $O/bench_$S.json 2> $O/bench_$S.err || { tail -20 $O/bench_$S.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_$S.json $S
  done
fi
