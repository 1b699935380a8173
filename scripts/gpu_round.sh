# Round evidence, part A: the full GPU suite, smoke, and the c2 / c4 / c5 / c3-phantom bench lines with
# CPU baselines and dice_vs_ref.  Part B (PART=B): rocprofv3 kernel-trace stats of the c2, c4 and c5 bench
# commands and the separate FETCH_SIZE / WRITE_SIZE PMC passes of each (tools/pmc_traffic.py).  Part C
# (PART=C): the GPU suite on the bounds-checked debug library (PMU_LIB=debug: a test fails if any kernel
# recorded an index-bound violation).
# Output under gpurun_out/round/; scripts/collect_round.sh copies it into profiles/<round>/.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O
cd $R
if [ "${PART:-A}" = "A" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
  echo "tests exit=$rc" >> $O/tests_gpu.log
  tail -2 $O/tests_gpu.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/tests_gpu.log | head -20; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
  timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
  timeout -k 10 600 python bench.py --workload probunet > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
  timeout -k 10 900 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
  timeout -k 10 600 python bench.py --data phantom --no-cpu-baseline > $O/bench_c3_phantom.json 2> $O/bench_c3.err || exit $?
  for f in c2 c4 c5 c3_phantom; do cut -c 1-200 $O/bench_$f.json; done
  echo round-a-done
elif [ "${PART}" = "C" ]; then
  PMU_LIB=debug timeout -k 10 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests_gpu_debug.log 2>&1; rc=$?
  echo "tests exit=$rc" >> $O/tests_gpu_debug.log
  tail -2 $O/tests_gpu_debug.log
  exit $rc
else
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o bench -- python3 $R/bench.py --workload probunet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c4.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
  cd $R
  for wl in unet c5 probunet; do
    WL=$wl EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_$wl.log 2>&1 || exit $?
    cp gpurun_out/pmc_bench/pmc_traffic_$wl.json gpurun_out/pmc_bench/summary_$wl.txt $O/
    head -1 $O/summary_$wl.txt
  done
  echo round-b-done
fi
