# Round 4, step P: fp32 Winograd weight gradient without register spills (tid laundered in the DMA
# (The spill-free variant measured slower — kbench 10.53 vs 10.28 ms, c2 678.4 vs 684.0 — and is not kept.)
# staging: the 1024-thread kernel reloaded spilled per-lane sources with a vmcnt(0) before every DMA
# round) — wgrad tests, kbench over the c2 shapes and c2 / c4 step A/B against the parent commit.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepP; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q tests/test_wino_gpu.py tests/test_unet_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
PMU_LIB=prev timeout -k 10 300 python tools/kbench.py --ops wgrad_wino > $O/kb_prev_$i.txt 2>&1 || exit 1
timeout -k 10 300 python tools/kbench.py --ops wgrad_wino > $O/kb_new_$i.txt 2>&1 || exit 1
done
for i in 1 2; do
PMU_LIB=prev timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_prev_$i.json 2> $O/b.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_new_$i.json 2> $O/b.err || exit 1
done
grep -h TOTAL $O/kb_*.txt
for f in $O/bench_*.json; do echo "$(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['kernels'].get('pmu_conv3x3_wgrad_wino',{}).get('ms'))")"; done
