set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/convt; mkdir -p $O; cd $R
for e in ${EXPS:-0 1 2}; do
PMU_CONVT_EXP=$e timeout -k 10 120 python tools/kbench_convt.py --ops ${OPS:-fwd,dgrad,wgrad} > $O/e$e.txt 2>&1 || { tail -20 $O/e$e.txt; exit 1; }
echo "EXP=$e"; grep -v amdgpu.ids $O/e$e.txt
done
