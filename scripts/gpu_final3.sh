# Round-3 GPU pass: full GPU suite, c2 / c5 / c4 bench lines, c5 with bf16 z forced (A/B of the
# contract-breaking option), rocprof stats of c2 and c5 into gpurun_out/$1.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-final3}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -x > $O/tests_gpu.log 2>&1; rc=$?
tail -3 $O/tests_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
cut -c 1-200 $O/bench_c2.json
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c5.json
timeout -k 10 600 python -c "
import sys, runpy
sys.path.insert(0, 'probabilistic-multiplanar-unet_amd')
import pmu_hip.engine as e
e.CFG.bf16_z = True; e._BF16_Z_FORCED = True
sys.argv = ['bench.py', '--workload', 'c5', '--no-cpu-baseline', '--no-eval']
runpy.run_path('bench.py', run_name='__main__')
" > $O/bench_c5_zb.json 2> $O/bench_c5_zb.err || exit $?
cut -c 1-200 $O/bench_c5_zb.json
timeout -k 10 600 python bench.py --workload probunet --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
cut -c 1-200 $O/bench_c4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
echo done
