set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/rawab; mkdir -p $O; cd $R
PMU_RAW_BMT=256 timeout -k 10 300 python tools/kbench.py --ops fwd_raw,dgrad_raw --iters 10 > $O/k256.txt 2>&1 || exit $?
PMU_RAW_BMT=512 timeout -k 10 300 python tools/kbench.py --ops fwd_raw,dgrad_raw --iters 10 > $O/k512.txt 2>&1 || exit $?
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/kbench.py --only 128,128,128 --iters 3 --ops fwd_raw > $O/p$i.log 2>&1 || echo "pass $i failed"
done
cd $R && python3 tools/pmc_summary.py $(find gpurun_out/rawab -name "*counter_collection.csv") > $O/summary.txt
echo rawab-done
