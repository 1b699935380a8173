set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcw; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
         "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/kbench.py --only ${SHAPE:-128,128,128} --iters 3 --ops ${OPS:-wgrad_bf16} > $O/p$i.log 2>&1 || echo "pass $i failed"
done
cd $R && python3 tools/pmc_summary.py $(find gpurun_out/pmcw -name "*counter_collection.csv") > $O/summary.txt
echo pmcw-done
