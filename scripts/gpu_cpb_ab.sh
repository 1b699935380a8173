# Co-block passes A/B for the fp32 Winograd kernels: kbench over the c2 shapes at the default pass
# count, without passes (co blocks as concurrent workgroups sharing the operand through L2) and with
# more passes; FETCH/WRITE PMC of two shapes for default vs no passes.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/cpb; mkdir -p $O; cd $R
timeout -k 10 300 python tools/kbench.py --ops dgrad_w4,fwd_w2h > $O/kb_default.txt 2>&1 || exit $?
PMU_WINO4_CPB=1 PMU_WINO2H_CPB=1 timeout -k 10 300 python tools/kbench.py --ops dgrad_w4,fwd_w2h > $O/kb_cpb1.txt 2>&1 || exit $?
PMU_WINO4_MINWG=256 PMU_WINO2H_MINWG=256 timeout -k 10 300 python tools/kbench.py --ops dgrad_w4,fwd_w2h > $O/kb_minwg256.txt 2>&1 || exit $?
tail -2 $O/kb_default.txt $O/kb_cpb1.txt $O/kb_minwg256.txt
export TMPDIR=/tmp
for S in 256,64,64 64,256,256 32,512,512; do
  for CFG in default cpb1; do
    for C in FETCH_SIZE WRITE_SIZE; do
      if [ $CFG = cpb1 ]; then export PMU_WINO4_CPB=1 PMU_WINO2H_CPB=1; else unset PMU_WINO4_CPB PMU_WINO2H_CPB; fi
      timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${S}_${CFG}_$C -o run -- python3 tools/kbench.py --ops dgrad_w4,fwd_w2h --only $S --iters 2 > $O/pmc_${S}_${CFG}_$C.log 2>&1 || exit $?
    done
  done
done
unset PMU_WINO4_CPB PMU_WINO2H_CPB
echo cpb-done
