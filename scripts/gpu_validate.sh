# Parity tests of the conv/prob paths, per-shape conv timings, both bench lines, and a 2-rank
# rehearsal of bench.py's data-parallel path on one GPU (gloo: RCCL needs one device per rank).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/val; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests/test_unet_gpu.py tests/test_probunet_gpu.py -q -p no:cacheprovider -x > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/kbench.py --ops fwd,dgrad,wgrad --iters 5 > $O/kbench.txt 2>&1 || exit $?
grep TOTAL $O/kbench.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit $?
timeout -k 10 400 python bench.py --workload probunet --steps 5 --warmup 2 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit $?
cut -c 1-230 $O/c2.json; cut -c 1-230 $O/c4.json
PMU_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-kernel-timing > $O/dp2.json 2> $O/dp2.err || { tail -20 $O/dp2.err; exit 1; }
cut -c 1-230 $O/dp2.json
echo validate-done
