# Round 4, step M: LDS-staged LDS-DMA weight pack (one workgroup per co block x chunk) — pack and DMA
# (Both alternative packs measured slower than the per-element one, which is kept)
# conv tests, then the pack kernels' rocprof time inside the c5 step.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepM; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q tests/test_pack_gpu.py tests/test_bf16_gpu.py -k "pack or dma" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof.log 2>&1 || exit 1
grep -h "pack" $O/prof/c5_kernel_stats.csv | cut -c1-160
