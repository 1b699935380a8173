set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu.log
tail -2 $O/tests_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
