# bf16 kernel parity + per-shape timings (fp32 reference lines for comparison).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bf16; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_bf16_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py --ops ${OPS:-fwd_bf16,dgrad_bf16,fwd} --iters 10 > $O/kbench.txt 2>&1 || exit $?
cat $O/kbench.txt
echo bf16-done
