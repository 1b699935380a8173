# Round evidence, part A: HBM traffic per kernel (separate FETCH_SIZE / WRITE_SIZE rocprofv3 --pmc passes,
# tools/pmc_traffic.py) of the c2, c5 and c4 bench steps, then rocprofv3 kernel-trace stats of the three
# bench commands.  The traffic files are copied into the box's profiles/r03 so later bench lines cite them.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O
cd $R
WL=unet bash scripts/gpu_pmc_bench.sh > $O/pmc.log 2>&1 || exit $?
WL=c5 EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c5.log 2>&1 || exit $?
WL=probunet EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c4.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o bench -- python3 $R/bench.py --workload probunet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
head -4 $R/gpurun_out/pmc_bench/summary_unet.txt
echo evidence-a-done
