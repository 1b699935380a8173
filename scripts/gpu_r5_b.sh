# Round 5: bf16 activation gradients (*_dxb) and the LDS-DMA bf16 weight gradient.  New kernel tests
# first, then the full GPU suite, kbench of the weight gradients over the c5 shapes, then c5 bench A/B
# (dx storage, weight-gradient kernel) and a c5 rocprof kernel-stats pass.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5b; mkdir -p $O
cd $R
( while sleep 45; do date >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wgrad_dma_gpu.py tests/test_dxb_gpu.py > $O/new_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $O/new_tests.log | tail -60
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16,wgrad_bf16d > $O/kbench_wgrad_c5.txt 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --ops dgrad_w4b,dgrad_w2hb > $O/kbench_dgrad_c2.txt 2>&1 || exit $?
grep -E "TOTAL" $O/kbench_dgrad_c2.txt
grep -E "TOTAL" $O/kbench_wgrad_c5.txt
timeout -k 10 900 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests > $O/tests_gpu.log 2>&1; rc=$?
tail -5 $O/tests_gpu.log
[ $rc -ne 0 ] && exit $rc
for v in "PMU_DX_BF16=0 PMU_WGRAD_DMA=0" "PMU_DX_BF16=1 PMU_WGRAD_DMA=0" "PMU_DX_BF16=1 PMU_WGRAD_DMA=1" "PMU_DX_BF16=0 PMU_WGRAD_DMA=0" "PMU_DX_BF16=1 PMU_WGRAD_DMA=1"; do
  tag=$(echo $v | tr -d ' =_' )
  env $v timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$tag.json 2> $O/bench_c5_$tag.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_$tag.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['step_mfma_busy_frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python bench.py --data phantom --no-cpu-baseline > $O/bench_c3_phantom.json 2> $O/bench_c3.err || exit $?
python -c "import json;d=json.load(open('$O/bench_c3_phantom.json'));print('c3', d['value'], d.get('gather'))"
echo r5b-done
