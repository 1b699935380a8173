# c5 evidence after a c5-only kernel change: PMC traffic (copied into the box's profiles/r03 so the
# bench line cites it), rocprofv3 kernel-trace stats, then the default c5 bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O
cd $R
WL=c5 EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c5.log 2>&1 || exit $?
cp $R/gpurun_out/pmc_bench/pmc_traffic_c5.json $R/profiles/r03/pmc_traffic_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
cd $R
timeout -k 10 500 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c5.json
echo evidence-c5-done
