# (CPU side) copy the evidence of a finished `gpu_round.sh` call from gpurun_out/ into profiles/<round>/
set -eu
R=${1:?round dir, e.g. r02}
P=profiles/$R; G=gpurun_out/round; B=gpurun_out/pmc_bench
mkdir -p $P
cp $G/bench.json $P/bench_c2.json
cp $G/bench_c4.json $P/bench_c4_probunet.json
cp $G/bench_c5.json $P/bench_c5.json
cp $G/tests_gpu.log $P/tests_gpu.log
cp $G/smoke.log $P/smoke.log
cp $G/prof/bench_kernel_stats.csv $P/rocprof_kernel_stats_c2.csv
cp $G/prof_c4/bench_kernel_stats.csv $P/rocprof_kernel_stats_c4.csv
cp $G/prof_c5/bench_kernel_stats.csv $P/rocprof_kernel_stats_c5.csv
for W in unet c5 probunet; do
  if [ -f $B/pmc_traffic_$W.json ]; then cp $B/pmc_traffic_$W.json $P/; cp $B/summary_$W.txt $P/pmc_traffic_${W}_summary.txt; fi
done
ls -la $P
