# bf16 kernel + model parity, then c5 and c2-bf16 bench lines.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bf16m; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests/test_bf16_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cut -c 1-1500 $O/c5.json
timeout -k 10 300 python bench.py --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline > $O/c2bf16.json 2> $O/c2bf16.err || { tail -20 $O/c2bf16.err; exit 1; }
cut -c 1-600 $O/c2bf16.json
echo bf16m-done
