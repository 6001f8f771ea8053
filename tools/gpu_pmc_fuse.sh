#!/bin/bash
# VALU / wait counters of the exact loop's bandwidth kernels (the fused triple
# against the MID triple and the pass), 4096^2 procedural convergence:
#   tools/gpu_pmc_fuse.sh <tag> [variant under tools/abx ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
tag=$1; shift
O=gpurun_out/${tag}_pmc
mkdir -p $O
RX='jacobi3_fused|jacobi3_mid|seqnorm_tables|seqnorm_merge'
for v in tree "$@"; do
    lp=""; [ "$v" != tree ] && lp="$R/tools/abx/$v/libof2d.so"
    p=0
    for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
        p=$((p + 1))
        OF2D_LIB_PATH=$lp OF2D_CONV_CASE=procedural OF2D_CONV_ONLY=1 timeout -s KILL 120 \
            rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d "$R/$O/${v}_$p" -o c \
            -- python3 -u "$R/tools/time_convergence.py" 4096 1 > "$O/${v}_$p.log" 2>&1 || exit $?
    done
    python3 tools/pmc_kernel_avg.py $(find "$O/${v}_1" "$O/${v}_2" -name '*counter_collection.csv') | sed "s/^/$v /"
done
