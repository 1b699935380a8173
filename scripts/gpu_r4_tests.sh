# Round 4: the new parity tests first (c5 at batch 16, 512-edge fusion, pack invalidation, ragged
# max-pool partials), then the full GPU suite on the shipped library and on the bounds-checked debug
# library (scripts/gpu_tests_both.sh), then one c5 bench line (MFMA accounting of every entry).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4t; mkdir -p $O
cd $R
# heartbeat while the oracle steps of the batch-16 test run (each stage prints, but a fresh box's first
# torch import and the fp64 / fp32 steps can leave a minute or two between lines)
( while sleep 45; do date >> $O/heartbeat.txt; done ) & HB=$!
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  "tests/test_bf16_gpu.py::test_c5_geometry_bf16_step_vs_oracle_batch16" tests/test_data_gpu.py::test_fusion_512_edge_vs_restatement \
  tests/test_pack_gpu.py::test_data_write_needs_invalidate_packs "tests/test_bnr_gpu.py::test_maxpool2_bwd_bnr" tests/test_bnr_gpu.py::test_encoder_bwd_bnr > $O/new_tests.log 2>&1; rc=$?
kill $HB
echo "new tests exit=$rc" >> $O/new_tests.log
grep -E "PASSED|FAILED|C5_STEP|oracle|Error|assert" $O/new_tests.log | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_tests_both.sh || exit $?
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-400 $O/bench_c5.json
echo r4-tests-done
