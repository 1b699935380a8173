# Round 5: the DMA conv's channel-block rule A/B (experiments build, PMU_DMA_BN128=1: 128-channel
# workgroups for every conv of >= 128 outputs) — kbench over the c5 shapes and the c5 bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5n; mkdir -p $O
cd $R
for r in 0 1; do
  PMU_LIB=exp PMU_DMA_BN128=$r timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab > $O/kbench_dma_c5_bn128_$r.txt 2>&1 || exit $?
  echo "rule=$r"; grep TOTAL $O/kbench_dma_c5_bn128_$r.txt
done
for r in 0 1 0 1; do
  PMU_LIB=exp PMU_DMA_BN128=$r timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_bn128_$r.json 2> $O/bench_c5_bn128_$r.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_bn128_$r.json'));print('rule=$r', d['value'], d['ms_per_step'])"
done
echo r5n-done
