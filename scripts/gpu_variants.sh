set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_unet_gpu.py -q -x -p no:cacheprovider > $O/tv.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tv.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0; do
  PMU_CONV_VARIANT=$v timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad,wgrad > $O/kbv$v.log 2>&1 || exit $?
done
echo done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bv.json 2> $O/bv.err || exit $?
