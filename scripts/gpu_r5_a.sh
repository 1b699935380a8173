# Round 5, first call: the new GPU tests (bench --gpus 2 launcher, 512^3 fusion), then c3's phantom
# leg through the GPU slicer and c4 with its batch-32 CPU baseline.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5a; mkdir -p $O
cd $R
( while sleep 45; do date >> $O/heartbeat.txt; done ) & HB=$!
timeout -k 10 900 python -u -m pytest -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_dp_gpu.py tests/test_data_gpu.py::test_fusion_512_cubed_vs_restatement > $O/new_tests.log 2>&1; rc=$?
echo "new tests exit=$rc" >> $O/new_tests.log
grep -E "PASSED|FAILED|Error|assert" $O/new_tests.log | head -40
if [ $rc -ne 0 ]; then kill $HB; exit $rc; fi
timeout -k 10 600 python bench.py --data phantom --classes 1 > $O/bench_c3_phantom.json 2> $O/bench_c3.err || { kill $HB; exit 1; }
timeout -k 10 900 python bench.py --workload probunet > $O/bench_c4.json 2> $O/bench_c4.err || { kill $HB; exit 1; }
kill $HB
cut -c 1-400 $O/bench_c3_phantom.json; cut -c 1-300 $O/bench_c4.json
echo r5a-done
