# All GPU tests, then the c2 / c4 bench lines (no CPU leg) for a quick check of a change.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sb; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
tail -3 $O/tests_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $O/tests_gpu.log | head -20; exit $rc; fi
for WL in ${WLS:-unet probunet}; do
  timeout -k 10 400 python bench.py --workload $WL --no-cpu-baseline --no-eval > $O/bench_$WL.json 2> $O/bench_$WL.err || { tail -5 $O/bench_$WL.err; exit 1; }
  python - "$O/bench_$WL.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernels"]; r=d["roofline"]
top=sorted(k.items(), key=lambda x:-x[1]["ms"])[:8]
print(d["config"]["workload"][:3], "value", d["value"], "ms", d["ms_per_step"], "roof", r["kernel"], r["frac"])
print("   ", " | ".join(f"{n[4:]} {v['ms']}" for n,v in top))
PY
done
