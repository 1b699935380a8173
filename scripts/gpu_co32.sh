# A/B of the 1024-thread 64-channel F(2x2) blocks against 512-thread 32-channel blocks capped at 128 VGPRs
# (two per CU) on every c2 layer shape (experiments build, PMU_WINO2H_CO=32).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/co32; mkdir -p $O; cd $R
timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w2h --iters 10 > $O/co64.txt 2>&1 || exit $?
PMU_LIB=exp PMU_WINO2H_CO=32 timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w2h --iters 10 > $O/co32.txt 2>&1 || exit $?
paste <(grep -v amdgpu $O/co64.txt) <(grep -v amdgpu $O/co32.txt | awk '{print $(NF-4), $(NF-3)}')
