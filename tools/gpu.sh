#!/bin/bash
# One parameterised GPU-box runner: the named steps in order, each under its
# own time limit, logs in gpurun_out/<tag>_<step>.log; stops at the first
# step that fails (a fault, abort or time limit ends the call there).
#   tools/gpu.sh <tag> <step>...
# steps: tests (pytest -m gpu), sntests (Logger-norm tests), slabtests
#        (slab group / RCCL / ngpus tests), smoke, bench,
#        prof (rocprofv3 kernel stats of bench.py), benchdrv / profdrv (the
#        driver's bench command, and its kernel stats), conv (convergence-on
#        timings at 4096^2), convprof (their kernel trace + stats),
#        configs (bench_configs.py), ranks (ngpus timings), ranksprof (their
#        kernel trace, 8 ranks; ranksprofq16 with 16 hardware queues, which
#        the profiler's queue interception needs for multi-thread launches,
#        DESIGN.md §5), texprof / freshprof (kernel trace of the
#        texture pair's warm / fresh loops), snbench /
#        snprof (the Logger-norm harness: stage timings / kernel stats),
#        fluidtrace / fluidtracealt (config 4's kernel trace with the in-tree
#        library / tools/lib_alt.so, and its GPU idle time: tools/gpu_idle.py),
#        convlarge (convergence-on procedural pair at 8192^2 and 16384^2; with
#        CONV_ALT=<dir> also the library tools/abx/<dir>/libof2d.so),
#        mtprobe / mtprobeprof (tools/mt_launch_probe: the slab group's
#        multi-thread launch pattern without the library, plain / under the
#        kernel trace; q16: 16 hardware queues, one per stream; serial: the eight
#        streams fed from one host thread)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out
mkdir -p $O
tag=${1:?tag}; shift
run() {  # run <name> <seconds> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$O/${tag}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 8 "$O/${tag}_$name.log"
    return $rc
}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for s in "$@"; do
    case $s in
        tests) run tests 900 $PT -m gpu tests ;;
        sntests) run sntests 600 $PT tests/test_gpu_seqnorm.py tests/test_gpu_convergence.py ;;
        slabtests) run slabtests 900 $PT tests/test_gpu_slab_local.py tests/test_gpu_rccl.py tests/test_gpu_ranks.py ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${tag}_prof" -o k -- python3 "$R/bench.py" --no-cpu-baseline ;;
        benchdrv) run benchdrv 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
        profdrv) run profdrv 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${tag}_profdrv" -o k -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-default-semantics ;;
        conv) run conv 600 python -u tools/time_convergence.py 4096 3 ;;
        convprof) run convprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${tag}_convprof" -o k -- python3 -u "$R/tools/time_convergence.py" 4096 1 ;;
        configs) run configs 900 python -u bench_configs.py ;;
        ranks) run ranks 600 python -u tools/time_ranks.py ;;
        ranksprof) OF2D_MAPS_DUMP="$R/$O/${tag}_ranksprof_maps.txt" run ranksprof 600 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_ranksprof" -o k -- python3 -u "$R/tools/time_ranks.py" 4096 1 fixed,conv 8 ;;
        ranksprofq16) GPU_MAX_HW_QUEUES=16 run ranksprofq16 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${tag}_ranksprofq16" -o k -- python3 -u "$R/tools/time_ranks.py" 4096 1 fixed,conv 8 ;;
        texprof) OF2D_CONV_CASE=texture OF2D_CONV_ONLY=1 run texprof 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_texprof" -o k -- python3 -u "$R/tools/time_convergence.py" 4096 1 ;;
        freshprof) OF2D_CONV_FRESH=1 OF2D_CONV_CASE=texture OF2D_CONV_ONLY=1 run freshprof 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_freshprof" -o k -- python3 -u "$R/tools/time_convergence.py" 4096 1 ;;
        snbench) run snbench 300 bash -c "tools/seqnorm_bench 4096 12 3 0.95 && tools/seqnorm_bench 4096 12 1 0.95 && tools/seqnorm_bench 4096 12 3 0.8" ;;
        snws) run snws 300 env SNB_WS=1 tools/seqnorm_bench 4096 12 3 0.95 ;;
        sndebug) OF2D_CONV_FRESH=1 OF2D_CONV_CASE=texture OF2D_CONV_ONLY=1 run sndebug 300 env OF2D_LIB_PATH=tools/abx/sndebug/libof2d.so python -u tools/time_convergence.py 4096 1 ;;  # tools/build_variant.sh sndebug registration.cpp -DOF2D_SN_DEBUG=1
        snprof) run snprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${tag}_snprof" -o k -- "$R/tools/seqnorm_bench" 4096 24 3 ;;
        fluidtrace) run fluidtrace 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_fluidtrace" -o k -- python3 -u "$R/bench_configs.py" --configs 4 --no-cpu && python3 tools/gpu_idle.py "$O/${tag}_fluidtrace/k_kernel_trace.csv" sor_strip_kernel | tee -a "$O/${tag}_fluidtrace.log" ;;
        fluidtracealt) OF2D_LIB_PATH="$R/tools/lib_alt.so" run fluidtracealt 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_fluidtracealt" -o k -- python3 -u "$R/bench_configs.py" --configs 4 --no-cpu && python3 tools/gpu_idle.py "$O/${tag}_fluidtracealt/k_kernel_trace.csv" sor_strip_kernel | tee -a "$O/${tag}_fluidtracealt.log" ;;
        convlarge) for n in 8192 16384; do for v in tree $CONV_ALT; do lp=""; [ $v != tree ] && lp="$R/tools/abx/$v/libof2d.so"; echo "== $n $v" >> "$O/${tag}_convlarge.log"; OF2D_LIB_PATH=$lp OF2D_CONV_CASE=procedural OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py $n 1 >> "$O/${tag}_convlarge.log" 2>&1 || exit $?; done; done; cat "$O/${tag}_convlarge.log" ;;
        mtprobe) run mtprobe 120 tools/mt_launch_probe 8 3000 ;;
        mtprobeprofserial) run mtprobeprofserial 180 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_mtprobeprofserial" -o k -- "$R/tools/mt_launch_probe" 8 3000 64 serial ;;
        mtprobeprofq16) GPU_MAX_HW_QUEUES=16 run mtprobeprofq16 180 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_mtprobeprofq16" -o k -- "$R/tools/mt_launch_probe" 8 3000 ;;
        mtprobeprof) MT_PROBE_MAPS="$R/$O/${tag}_mtprobeprof_maps.txt" run mtprobeprof 180 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/${tag}_mtprobeprof" -o k -- "$R/tools/mt_launch_probe" 8 3000 ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac || exit $?
done
echo ALL-DONE
