# Round 5: c5 with bf16 activation gradients + the LDS-DMA weight gradient: A/B bench lines, rocprof
# kernel stats, PMC traffic of the step.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5e; mkdir -p $O
cd $R
for v in "PMU_DX_BF16=0 PMU_WGRAD_DMA=0" "PMU_DX_BF16=1 PMU_WGRAD_DMA=1" "PMU_DX_BF16=0 PMU_WGRAD_DMA=0" "PMU_DX_BF16=1 PMU_WGRAD_DMA=1"; do
  tag=$(echo $v | tr -d ' =_' )
  env $v timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$tag.json 2> $O/bench_c5_$tag.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_$tag.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['step_mfma_busy_frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
cd $R
WL=c5 EXTRA=--no-eval bash scripts/gpu_pmc_bench.sh > $O/pmc_c5.log 2>&1 || exit $?
tail -3 $O/pmc_c5.log
cp gpurun_out/pmc_bench/pmc_traffic_c5.json gpurun_out/pmc_bench/summary_c5.txt $O/
echo r5e-done
