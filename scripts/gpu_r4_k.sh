# Round 4, step K: 6-wave bf16 weight gradient (one co group, 4 co fragments per wave; PMU_WGB6=1)
# (The 6-wave variant was 2.0x slower over the c5 shapes and is not kept)
# against the 12-wave default — parity of the variant, then kbench over the c5 shapes, both orders.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stepK; mkdir -p $O
cd $R
PMU_WGB6=1 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q tests/test_bf16_gpu.py -k "wgrad" > $O/tests_wgb6.log 2>&1 || { tail -30 $O/tests_wgb6.log; exit 1; }
tail -1 $O/tests_wgb6.log
timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16 > $O/kb_default.txt 2>&1 || exit 1
PMU_WGB6=1 timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16 > $O/kb_wgb6.txt 2>&1 || exit 1
timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16 > $O/kb_default2.txt 2>&1 || exit 1
grep TOTAL $O/kb_*.txt
