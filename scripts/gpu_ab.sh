# A/B/... of an env switch on kbench ops over the c2 shapes: VAR=name VALS="a b c" OPS=... [TESTS=...]
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
for v in $VALS; do
  if [ -n "${TESTS:-}" ]; then
    env $VAR=$v timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
    echo "$VAR=$v: $(tail -1 $O/tests_$v.log)"
  fi
  env $VAR=$v timeout -k 10 300 python tools/kbench.py --ops $OPS --iters ${ITERS:-10} > $O/kb_$v.log 2>&1 || exit $?
done
for v in $VALS; do echo "== $VAR=$v"; grep -E "^(fwd|dgrad|wgrad|TOTAL)" $O/kb_$v.log | awk '{printf "%s %s %s %s | ", $1,$2,$3,$(NF-4)} END {print ""}' ; grep TOTAL $O/kb_$v.log; done
