# Round 4, step Q: 4-wave LDS-DMA ConvT workgroups (BM 128, three stages in 72 KB: two per CU, one's
# (The 4-wave variant measured equal — ConvT forward -4%, input gradient +3% in kbench, c5 step within noise — and is not kept.)
# epilogue under the other's loads / MFMAs; PMU_CONVT_W4=1) against the 8-wave default — ConvT tests
# with the variant, kbench over the c5 decoder shapes, c5 step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepQ; mkdir -p $O
cd $R
PMU_CONVT_W4=1 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q tests/test_convT_gpu.py tests/test_bf16_gpu.py -k "convT or c5_geometry_bf16_step_vs_oracle and not batch16" > $O/tests_w4.log 2>&1 || { tail -30 $O/tests_w4.log; exit 1; }
tail -1 $O/tests_w4.log
for i in 1 2; do
timeout -k 10 300 python tools/kbench_convt.py --c5 --ops fwd_dma,dgrad_dma > $O/kb_w8_$i.txt 2>&1 || exit 1
PMU_CONVT_W4=1 timeout -k 10 300 python tools/kbench_convt.py --c5 --ops fwd_dma,dgrad_dma > $O/kb_w4_$i.txt 2>&1 || exit 1
done
for i in 1 2; do
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_w8_$i.json 2> $O/b.err || exit 1
PMU_CONVT_W4=1 timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_w4_$i.json 2> $O/b.err || exit 1
done
grep -h TOTAL $O/kb_*.txt
for f in $O/bench_*.json; do echo "$(basename $f) $(python -c "import json; d=json.load(open('$f')); k=d['kernels']; print(d['value'], d['ms_per_step'], {n: v['ms'] for n, v in k.items() if 'convT2x2' in n and ('dma' in n)})")"; done
