# Per-shape HBM traffic of kbench ops beside their algorithmic bytes (tools/pmc_shapes.py): for each op of
# OPS (','-separated) a timing run, then one rocprofv3 --pmc pass each for FETCH_SIZE and WRITE_SIZE.
#   OPS=mat_bnrelu,mat_bnbwd_xb KERNEL=frame_stream_kernel KB_EXTRA="--c5" N=16 bash scripts/gpu_pmc_shapes.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcs; mkdir -p $O; cd $R
export TMPDIR=/tmp
IT=${ITERS:-3}
IFS=',' read -ra OS <<< "$OPS"
for op in "${OS[@]}"; do
  timeout -k 10 300 python tools/kbench.py --ops $op --iters 10 ${KB_EXTRA:-} > $O/time_$op.txt 2>&1 || { tail -5 $O/time_$op.txt; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $O/${op}_$C -o p --output-format csv -- python3 tools/kbench.py --ops $op --iters $IT ${KB_EXTRA:-} > $O/${op}_$C.log 2>&1 || exit $?
  done
  python3 tools/pmc_shapes.py $O/${op}_FETCH_SIZE $O/${op}_WRITE_SIZE $KERNEL $IT --N ${N:-32} --op $op ${KB_EXTRA:-} > $O/shapes_$op.txt || exit $?
  cat $O/shapes_$op.txt
  grep TOTAL $O/time_$op.txt
done
echo pmc-shapes-done
