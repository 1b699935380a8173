set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/w2order; mkdir -p $O; cd $R
for cfg in "0:0" "1:0" "0:1" "1:1"; do
  o=${cfg%%:*}; c=${cfg##*:}
  if [ "$c" = "1" ]; then export PMU_WINO2H_CPB=1; else unset PMU_WINO2H_CPB; fi
  PMU_LIB=exp PMU_WINO2H_ORDER=$o timeout -k 10 200 python tools/kbench.py --ops fwd_w2h --iters 10 > $O/o$o$c.txt 2>&1 || { tail -20 $O/o$o$c.txt; exit 1; }
  echo "ORDER=$o CPB1=$c"; grep -v amdgpu.ids $O/o$o$c.txt
done
