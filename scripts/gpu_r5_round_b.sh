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
# c4 A/B of the pooled-gradient fusion (fp32 parts)
cd $R
for f in 0 1 0 1; do
  PMU_POOL_FUSE=$f timeout -k 10 600 python bench.py --workload probunet --no-cpu-baseline > $O/bench_c4_fuse$f.json 2> $O/bench_c4_fuse$f.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c4_fuse$f.json'));print('c4 pool_fuse=$f', d['value'], d['ms_per_step'])"
done
echo round-b2-done
