# Round 4, step O: per-shape HBM bytes of the F(4x4) BN-backward input gradient over the c2 layer
# shapes (kbench dgrad_w4b, batch 32) against its algorithmic bytes — two separate --pmc passes.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepO; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$C -o run -- python3 $R/tools/kbench.py --ops dgrad_w4b --iters 3 > $O/$C.log 2>&1 || exit 1
done
python3 $R/tools/pmc_shapes.py $O/FETCH_SIZE $O/WRITE_SIZE conv3x3_wino4_kernel 3 > $O/w4b_shapes.txt || exit 1
cat $O/w4b_shapes.txt
