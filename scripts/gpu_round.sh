# Round evidence in one call: all GPU tests, smoke, c2 / c4 / c5 bench lines (with CPU baselines and
# dice_vs_ref), rocprofv3 kernel-trace stats of the c2, c4 and c5 bench commands, and the separate
# FETCH_SIZE / WRITE_SIZE PMC passes of c2, c5 and c4 (tools/pmc_traffic.py).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu.log
tail -2 $O/tests_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 python bench.py --workload probunet > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 900 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o bench -- python3 $R/bench.py --workload probunet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c4.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
cd $R
WL=unet bash scripts/gpu_pmc_bench.sh > $O/pmc.log 2>&1 || exit $?
WL=c5 EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c5.log 2>&1 || exit $?
WL=probunet EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c4.log 2>&1 || exit $?
cut -c 1-300 $O/bench.json; cut -c 1-300 $O/bench_c4.json; cut -c 1-300 $O/bench_c5.json
echo round-done
