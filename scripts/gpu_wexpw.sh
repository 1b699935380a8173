set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wexpw; mkdir -p $O; cd $R
for e in ${EXPS:-0 1 3}; do
PMU_WINO_EXP=$e timeout -k 10 120 python tools/kbench.py --ops wgrad_wino --only ${SHAPE:-32,512,512} --iters 10 > $O/e$e.txt 2>&1 || exit $?
echo "EXP=$e $(grep TOTAL $O/e$e.txt)"
done
