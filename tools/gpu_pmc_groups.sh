#!/bin/bash
# Per-kernel SQ counters of a secondary configuration, in groups of <= 8 SQ
# counters per rocprofv3 pass (kernel trace only, one pass per group):
#   bash tools/gpu_pmc_groups.sh <tag> <bench_configs.py args...>
# e.g.  bash tools/gpu_pmc_groups.sh demons --configs 3 --iters 5
# Writes gpurun_out/pmc_<tag>/summary.txt (average value per kernel launch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
TAG=$1
shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
n=0
for grp in "$G1" "$G2"; do
  n=$((n + 1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/g$n" -o c -- python3 "$R/bench_configs.py" "$@" > $OUT/g$n.log 2>&1
  rc=$?
  echo "group $n rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, os, sys
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/g*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0][:70], r.get("Dispatch_Id", ""))
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, v in d.items():
            out[k][c].append(v)
with open(sys.argv[1] + "/summary.txt", "w") as fh:
    for k, d in out.items():
        fh.write(k + "\n    " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())) + "\n")
print(open(sys.argv[1] + "/summary.txt").read())
PY
