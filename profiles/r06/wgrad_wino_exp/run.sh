set -u
O=gpurun_out/r6z; mkdir -p $O
for v in 0 1 3 0 1 3; do
  PMU_LIB=exp PMU_WINO_EXP=$v timeout -k 10 300 python tools/kbench.py --ops wgrad_wino --iters 10 > $O/kb_exp$v.log 2>&1 || exit $?
  echo "exp=$v $(grep TOTAL $O/kb_exp$v.log)"
done
