set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_unet_gpu.py -q -x -p no:cacheprovider > $O/tq.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tq.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py --ops ${OPS:-fwd,dgrad,wgrad} > $O/kbq.log 2>&1 || exit $?
if [ "${BENCH:-1}" = "1" ]; then timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bq.json 2> $O/bq.err || exit $?; fi
echo done
