set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/test_unet_gpu.py -q -p no:cacheprovider > $O/t2.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/prof1.log 2>&1
echo "prof exit=$?"
