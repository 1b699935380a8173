# HBM traffic of every kernel of the bench step: two separate rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE; they cannot share a pass on gfx950), kernel-trace only, CSV output.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_bench; mkdir -p $O
WL=${WL:-unet}
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$C -o run -- python3 $R/bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing ${EXTRA:-} > $O/$C.log 2>&1 || exit $?
done
python3 $R/tools/pmc_traffic.py $O/FETCH_SIZE $O/WRITE_SIZE $O/pmc_traffic_$WL.json --steps 3 > $O/summary_$WL.txt || exit $?
cat $O/summary_$WL.txt
echo pmc-bench-done
