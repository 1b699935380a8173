# Selected GPU test files (args), verbose, with the c5 Dice-gap JSON line kept.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/nt; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v -s -m gpu -p no:cacheprovider --timeout 400 --timeout-method thread "$@" > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc" >> $O/tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed|C5_DICE_GAP" $O/tests.log | tail -40
exit $rc
