# MFMA counter calibration (round-4 verdict item 5): SQ_VALU_MFMA_BUSY_CYCLES and the MFMA
# instruction / math-op counters of kernels whose executed MFMA work is known from the launch
# (tools/kbench.py, one shape, batch N = 1, 4, 16), one rocprofv3 --pmc pass per run.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/mfma; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for N in 1 4 16; do
  for S in 256,64,64 64,512,512; do
    T=n${N}_$(echo $S | tr , _)
    timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/$T -o run -- python3 $R/tools/kbench.py --only $S --N $N --ops fwd_w2h,fwd_dma,wgrad_bf16,dgrad_w4 --iters 1 > $O/$T.log 2>&1 || exit $?
    echo "$T done"
  done
done
python3 $R/tools/mfma_calib.py $O > $O/summary.txt || exit $?
cat $O/summary.txt
