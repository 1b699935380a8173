# Row e rehearsal on one GPU: overlapped bucket all-reduce (gloo, 2 ranks on cuda:0) and bench N=2.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dp; mkdir -p $O; cd $R
export PMU_DIST_BACKEND=gloo
timeout -k 10 240 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 280 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
for wl in unet probunet; do
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 2 --steps 3 --warmup 1 --workload $wl --batch 4 --no-cpu-baseline --no-kernel-timing > $O/bench_$wl.log 2>&1 || { tail -40 $O/bench_$wl.log; exit 1; }
grep '"metric"' $O/bench_$wl.log | cut -c1-200
done
