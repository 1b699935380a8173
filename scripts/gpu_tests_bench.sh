# GPU tests (new parity tests first), smoke, and the default c2 bench line with dice_vs_ref.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tb; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_train_gpu.py tests/test_unet_gpu.py tests/test_probunet_gpu.py tests/test_dp_gpu.py > $O/tests_new.log 2>&1
rc=$?; echo "new tests exit=$rc" >> $O/tests_new.log; tail -3 $O/tests_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1
rc2=$?; echo "tests exit=$rc2" >> $O/tests_gpu.log; tail -3 $O/tests_gpu.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c 1-400 $O/bench.json
