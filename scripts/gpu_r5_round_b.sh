# Round 5 evidence, part B: rocprofv3 kernel-trace stats of the c2 / c4 / c5 bench commands and the
# separate FETCH_SIZE / WRITE_SIZE PMC passes of each (tools/pmc_traffic.py).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round5; mkdir -p $O
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
