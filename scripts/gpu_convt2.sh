set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/convt; mkdir -p $O; cd $R
timeout -k 10 200 python -u -m pytest tests/test_convT_gpu.py tests/test_unet_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 120 python tools/kbench_convt.py --ops fwd,dgrad,wgrad > $O/k.txt 2>&1 || { tail -20 $O/k.txt; exit 1; }
grep -v amdgpu.ids $O/k.txt
