# SQ counters of the c5 transposed-conv kernels (tools/kbench_convt.py --c5), one rocprofv3 --pmc pass
# per counter set; summary per kernel into gpurun_out/pmcconvt/summary.txt.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcconvt; mkdir -p $O; cd $R
export TMPDIR=/tmp
PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
IFS=';' read -ra PS <<< "$PASSES"
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $O/p$i -o p$i --output-format csv -- python tools/kbench_convt.py --c5 --ops fwd_dma,dgrad_dma,wgrad_bf16 --iters 3 > $O/p$i.log 2>&1 || exit $?
done
python tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.txt
cat $O/summary.txt
