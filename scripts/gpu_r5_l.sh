# Round 5: c2 A/B of the unstored head gradient (PMU_HEAD_FUSE=0/1, alternating, 3 each), then a c5
# rocprof kernel-stats pass of the current code.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5l; mkdir -p $O
cd $R
for i in 1 2 3; do
  for f in 0 1; do
    PMU_HEAD_FUSE=$f timeout -k 10 600 python bench.py --no-cpu-baseline --steps 20 > $O/bench_c2_head${f}_$i.json 2> $O/bench_c2_head${f}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c2_head${f}_$i.json'));print('c2 head_fuse=$f', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o bench -- python3 $R/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-eval > $O/prof_c5.log 2>&1 || exit $?
echo r5l-done
