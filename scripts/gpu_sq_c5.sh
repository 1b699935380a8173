# SQ counters of c5 kernels (tools/kbench.py --c5 ops) on a list of shapes, two rocprofv3 --pmc passes
# each, summarised per kernel (tools/pmc_summary.py).
#   OPS     kbench ops (default fwd_dma,dgrad_dma; the weight gradients: wgrad_bf16,wgrad_bf16d)
#   SHAPES  space-separated H,Cin,Cout (default "512,64,64 64,512,512")
#   TAG     output directory under gpurun_out/ (default sq_c5)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-sq_c5}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU GRBM_COUNT"
for S in ${SHAPES:-512,64,64 64,512,512}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    T=$(echo $S | tr , _)_p$i
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/$T -o run -- python3 $R/tools/kbench.py --c5 --only $S --ops ${OPS:-fwd_dma,dgrad_dma} --iters 2 > $O/$T.log 2>&1 || exit $?
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*$(echo $S | tr , _)_p*" -name "*counter_collection.csv") > $O/summary_$(echo $S | tr , _).txt || exit $?
  cat $O/summary_$(echo $S | tr , _).txt
done
