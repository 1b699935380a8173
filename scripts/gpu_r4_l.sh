# Round 4, step L: bf16 LDS-DMA ConvT forward decodes a fragment's pixel once (W % 32 == 0) instead of
# two integer divisions per store — ConvT tests, kbench over the c5 decoder shapes and c5 step A/B
# against the previous library (PMU_LIB=prev, built from the parent commit).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepL; mkdir -p $O
cd $R
T="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T -q tests/test_convT_gpu.py tests/test_bf16_gpu.py -k "convT or dma or c5_geometry_bf16_step_vs_oracle and not batch16" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
PMU_LIB=prev timeout -k 10 300 python tools/kbench_convt.py --c5 --ops fwd > $O/kb_prev_$i.txt 2>&1 || exit 1
timeout -k 10 300 python tools/kbench_convt.py --c5 --ops fwd > $O/kb_new_$i.txt 2>&1 || exit 1
done
for i in 1 2; do
PMU_LIB=prev timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_prev_$i.json 2> $O/b.err || exit 1
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_new_$i.json 2> $O/b.err || exit 1
done
grep -h TOTAL $O/kb_*.txt
for f in $O/bench_*.json; do echo "$(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'])")"; done
