# Round 4, step N: F(4x4) input-gradient co-block passes per workgroup — c2 step A/B over
# PMU_WINO4_MINWG (the workgroup floor that caps the passes; 1024 default).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepN; mkdir -p $O
cd $R
for i in 1 2; do
for m in 1024 4096 256; do
PMU_WINO4_MINWG=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_minwg${m}_$i.json 2> $O/b.err || exit 1
done
done
for f in $O/bench_*.json; do echo "$(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['kernels'].get('pmu_conv3x3_dgrad_wino4_bnr',{}).get('ms'), d['kernels'].get('pmu_conv3x3_dgrad_wino4',{}).get('ms'))")"; done
