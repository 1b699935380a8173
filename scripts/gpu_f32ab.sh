set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/f32ab; mkdir -p $O; cd $R
PMU_CONV_IMPL=pipe2 timeout -k 10 300 python -m pytest tests/test_unet_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad --iters 10 > $O/k1.txt 2>&1 || exit $?
PMU_CONV_IMPL=pipe2 timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad --iters 10 > $O/k2.txt 2>&1 || exit $?
grep TOTAL $O/k1.txt $O/k2.txt
PMU_CONV_IMPL=pipe2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/c2.json 2> $O/c2.err || exit 1
cut -c 1-200 $O/c2.json
