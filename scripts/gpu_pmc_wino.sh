set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcw; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1 -o p1 --output-format csv -- python tools/kbench.py --ops ${OPS:-fwd_wino,fwd} --only ${SHAPE:-32,512,512} --iters 2 > $O/p1.log 2>&1 || exit $?
find $O/p1 -name "*counter_collection.csv" | head -1 > $O/files.txt
python - <<'PY'
import csv, collections, os
O=os.environ.get("GRAFT_REPO_ROOT")+"/gpurun_out/pmcw"
f=open(O+"/files.txt").read().strip()
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
for r in csv.DictReader(open(f)):
    k=r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]]+=float(r["Counter_Value"])
    cnt[(k,r["Counter_Name"])]+=1
for k,d in agg.items():
    print(k)
    for c,v in sorted(d.items()): print(f"   {c:28s} {v/cnt[(k,c)]:.4g}")
PY
