set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_unet_gpu.py -q -p no:cacheprovider > $O/t3.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/t3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py > $O/kbench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || exit $?
echo done
