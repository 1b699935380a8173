# Bench-line A/B over env settings: SETS="VAR=a,VAR2=b VAR=c" (comma-joined assignments per set), WL=unet|c5|probunet
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bab; mkdir -p $O; cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
i=0
for S in $SETS; do
  i=$((i+1))
  env $(echo $S | tr ',' ' ') timeout -k 10 400 python bench.py --workload ${WL:-unet} --no-cpu-baseline --no-eval --steps ${STEPS:-10} > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$S" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernels"]
top=sorted(k.items(), key=lambda x:-x[1]["ms"])[:8]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], " | ".join(f"{n[4:]} {v['ms']}" for n,v in top))
PY
done
