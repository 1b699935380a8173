# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes, kernel-trace only) of the c2, c5 and c4 bench steps.
set -u
R=$GRAFT_REPO_ROOT
for WL in unet c5 probunet; do
  O=$R/gpurun_out/pmc_r03/$WL; mkdir -p $O
  cd /tmp && export TMPDIR=/tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$C -o run -- python3 $R/bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-eval > $O/$C.log 2>&1 || exit $?
  done
  python3 $R/tools/pmc_traffic.py $O/FETCH_SIZE $O/WRITE_SIZE $O/pmc_traffic_$WL.json > $O/summary_$WL.txt || exit $?
  head -12 $O/summary_$WL.txt
done
echo pmc-done
