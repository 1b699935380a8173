# c2 / c5 bench lines and rocprof kernel stats (one short profiled run each) into gpurun_out/$1.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-quick}; mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
cut -c 1-200 $O/bench_c2.json
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
echo done
