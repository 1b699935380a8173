set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wino; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py tests/test_tee32_gpu.py tests/test_unet_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --ops fwd,fwd_wino,dgrad,dgrad_wino --iters 10 > $O/k.txt 2>&1 || exit $?
grep TOTAL $O/k.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
cut -c 1-300 $O/c2.json
