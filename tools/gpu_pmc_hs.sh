#!/bin/bash
# SQ issue counters of HS triple-kernel variants (tools/hs_gi_ab PMC mode), in
# groups of <= 8 SQ counters per rocprofv3 pass (kernel trace only):
#   bash tools/gpu_pmc_hs.sh <tag> <variant index>... 
# Writes gpurun_out/pmc_hs_<tag>/summary.txt (average per launch per kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
TAG=$1
shift
OUT=gpurun_out/pmc_hs_$TAG
mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
for v in "$@"; do
  n=0
  for grp in "$G1" "$G2"; do
    n=$((n + 1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/v${v}_g$n" -o c -- "$R/tools/hs_gi_ab" 4096 30 1 $v > $OUT/v${v}_g$n.log 2>&1
    rc=$?
    echo "variant $v group $n rc=$rc"
    [ $rc -le 1 ] || exit $rc
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/v*_g*/**/*counter_collection.csv", recursive=True)):
    v = f.split("/v")[1].split("_g")[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        key = ("v" + v + " " + r["Kernel_Name"].split("(")[0][:60], r.get("Dispatch_Id", ""))
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, val in d.items():
            out[k][c].append(val)
with open(sys.argv[1] + "/summary.txt", "w") as fh:
    for k, d in sorted(out.items()):
        fh.write(k + "\n    " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())) + "\n")
print(open(sys.argv[1] + "/summary.txt").read())
PY
