#!/bin/bash
# Per-kernel PMC counters of a secondary configuration (default: Demons, cfg3),
# one counter per rocprofv3 pass (kernel trace only).
#   bash tools/gpu_pmc_cfg.sh [config]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
CFG=${1:-3}
mkdir -p gpurun_out/pmc_cfg
for c in ${PMC_COUNTERS:-FETCH_SIZE WRITE_SIZE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD}; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_cfg/$c" -o c -- python3 "$R/bench_configs.py" --configs $CFG --iters 5 > gpurun_out/pmc_cfg/$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections, os
out = collections.defaultdict(dict)
for d in sorted(glob.glob("gpurun_out/pmc_cfg/*/")):
    c = os.path.basename(d.rstrip("/"))
    f = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        acc[r["Kernel_Name"].split("(")[0][:60]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        out[k][c] = sum(v) / len(v)
with open("gpurun_out/pmc_cfg/summary.txt", "w") as fh:
    for k, d in out.items():
        fh.write(k + "  " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())) + "\n")
print(open("gpurun_out/pmc_cfg/summary.txt").read())
PY
