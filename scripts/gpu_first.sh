set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/first; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_unet_gpu.py tests/test_probunet_gpu.py tests/test_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2>$O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $O/c5.json 2>$O/c5.err || { tail $O/c5.err; exit 1; }
python - <<'P'
import json
for f in ["gpurun_out/first/c2.json", "gpurun_out/first/c5.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    print(f, d["value"], {n: k[n]["ms"] for n in k if "first" in n}, d.get("c5_volume_fusion_eval", {}).get("predict_slices_per_s"))
P
