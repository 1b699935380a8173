# fp32 conv: pipelined (default) vs 2-block kernel (PMU_CONV_IMPL=sync), parity of both, then the c2 bench with each.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/f32p; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_unet_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
if [ $rc -ne 0 ]; then tail -40 $O/tests.log; exit $rc; fi
timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad --iters 10 > $O/kb_pipe.txt 2>&1 || exit $?
PMU_CONV_IMPL=sync timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad --iters 10 > $O/kb_cls.txt 2>&1 || exit $?
grep TOTAL $O/kb_pipe.txt $O/kb_cls.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c2p.json 2> $O/c2p.err || exit 1
cut -c 1-300 $O/c2p.json
echo f32p-done
