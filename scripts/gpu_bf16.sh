# bf16 kernel parity + per-shape timings (A/B: PMU_BF16_NOPIPE=1 selects the synchronous kernel).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bf16; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_bf16_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then tail -40 $O/tests.log; exit $rc; fi
timeout -k 10 300 python tools/kbench.py --ops ${OPS:-fwd_bf16,dgrad_bf16} --iters 10 > $O/kbench.txt 2>&1 || exit $?
grep TOTAL $O/kbench.txt
if [ "${AB:-0}" = "1" ]; then
PMU_BF16_NOPIPE=1 timeout -k 10 300 python tools/kbench.py --ops ${OPS:-fwd_bf16,dgrad_bf16} --iters 10 > $O/kbench_nopipe.txt 2>&1 || exit $?
grep TOTAL $O/kbench_nopipe.txt
fi
if [ "${C5:-0}" = "1" ]; then
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cut -c 1-400 $O/c5.json
fi
echo bf16-done
