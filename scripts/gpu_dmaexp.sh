set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dmaexp; mkdir -p $O; cd $R
for sh in ${SHAPES:-512,64,64 512,128,64}; do
for ed in ${SETS:-0:0 1:0 2:0 3:0}; do
  e=${ed%%:*}; d=${ed##*:}
  PMU_LIB=exp PMU_DMA_EXP=$e PMU_DMA_DELAY=$d timeout -k 10 120 python tools/kbench.py --c5 --ops fwd_dma --only $sh --iters 20 > $O/e.txt 2>&1 || { tail -20 $O/e.txt; exit 1; }
  echo "EXP=$e DELAY=$d $(grep 'fwd_dma H' $O/e.txt)"
done
done
