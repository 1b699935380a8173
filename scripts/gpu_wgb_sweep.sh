set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wgb; mkdir -p $O; cd $R
for b in 256 512 128 1024; do
  PMU_WGB_BLOCKS=$b timeout -k 10 200 python tools/kbench.py --c5 --ops wgrad_bf16 --iters 10 > $O/b$b.txt 2>&1 || { tail -20 $O/b$b.txt; exit 1; }
  echo "BLOCKS=$b"; grep -v amdgpu.ids $O/b$b.txt
done
