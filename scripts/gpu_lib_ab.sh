# Bench A/B of two builds of the library: LIB_B (a file next to libpmunet_hip.so) vs the default,
# for the workloads in WLS (unet | probunet | c5), STEPS steps each; per-kernel top list printed.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/libab; mkdir -p $O; cd $R
D=probabilistic-multiplanar-unet_amd/pmu_hip
cp $D/libpmunet_hip.so $O/lib_a.so
for V in a b; do
  if [ $V = b ]; then cp $D/$LIB_B $D/libpmunet_hip.so; fi
  for W in ${WLS:-unet}; do
    timeout -k 10 400 python bench.py --workload $W --no-cpu-baseline --no-eval --steps ${STEPS:-10} > $O/${V}_$W.json 2> $O/${V}_$W.err || { tail -5 $O/${V}_$W.err; exit 1; }
    python - "$O/${V}_$W.json" "$V $W" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernels"]
top=sorted(k.items(), key=lambda x:-x[1]["ms"])[:10]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], " | ".join(f"{n[4:]} {v['ms']}" for n,v in top))
PY
  done
done
cp $O/lib_a.so $D/libpmunet_hip.so
