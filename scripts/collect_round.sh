# (CPU side) copy the evidence of finished `scripts/gpu_round.sh` calls (parts A and B) from gpurun_out/round
# into profiles/<round>/round/
set -eu
R=${1:?round dir, e.g. r06}
P=profiles/$R/round; G=gpurun_out/round
mkdir -p $P
for f in tests_gpu.log tests_gpu_debug.log smoke.log bench_c2.json bench_c4.json bench_c5.json bench_c3_phantom.json; do
  [ -f $G/$f ] && cp $G/$f $P/
done
for d in prof:c2 prof_c4:c4 prof_c5:c5; do
  src=${d%%:*}; tag=${d##*:}
  [ -f $G/$src/bench_kernel_stats.csv ] && cp $G/$src/bench_kernel_stats.csv $P/rocprof_kernel_stats_$tag.csv
done
for W in unet c5 probunet; do
  if [ -f $G/pmc_traffic_$W.json ]; then cp $G/pmc_traffic_$W.json $G/summary_$W.txt $P/; fi
done
ls -la $P
