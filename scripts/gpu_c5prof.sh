# c5 GEMM kernels: per-shape timings of the bf16 conv kernels, then SQ counters of the LDS-DMA conv
# on a deep and a shallow c5 layer.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c5prof; mkdir -p $O; cd $R
timeout -k 10 300 python tools/kbench.py --c5 --ops ${OPS:-fwd_dma,dgrad_dma,wgrad_bf16} --iters 5 > $O/kbench_c5.txt 2>&1 || exit $?
cat $O/kbench_c5.txt | tail -8
for SH in ${SHAPES:-64,512,512 512,64,64}; do
  OPS=${POPS:-fwd_dma} SHAPE=$SH KB_EXTRA="--c5" bash scripts/gpu_pmc_kernel.sh > $O/pmc_$SH.txt 2>&1 || exit $?
  cp gpurun_out/pmck/summary.txt $O/pmc_summary_$SH.txt
done
echo c5prof-done
