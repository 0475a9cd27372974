#!/bin/bash
# GPU-box measurement pass: bench (with the CPU baseline), rocprofv3 kernel
# stats, PMC passes (HBM bytes; SQ issue/wait counters; scratch / memory
# instruction counts), and the per-world forward latency histogram
# (-DNIMBLE_STAGE_TIMING build in dbg/).
# Usage: bash tools/gpu_measure.sh <tag> [bench args]
set -o pipefail
TAG=${1:-r02}
shift || true
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
B="python bench.py --no-cpu-baseline $*"
timeout -k 10 300 python bench.py "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCH FAILED; tail -20 $O/bench_$TAG.err; exit 1; }
cut -c1-2500 $O/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- $B --steps 20 --warmup 3 > $O/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof_$TAG.log; exit 1; }
echo PROF OK
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$TAG -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc1_$TAG.log 2>&1 || { echo PMC1 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_$TAG -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc2_$TAG.log 2>&1 || { echo PMC2 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $O/pmc_sq_$TAG -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc3_$TAG.log 2>&1 || { echo PMC3 FAILED; tail -5 $O/pmc3_$TAG.log; exit 1; }
echo PMC OK
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/stage_hist_$TAG.json timeout -k 10 120 python tools/stage_timing.py > $O/stage_$TAG.log 2>&1 || { echo STAGE FAILED; tail -20 $O/stage_$TAG.log; exit 1; }
tail -1 $O/stage_$TAG.log
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_FLAT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-trace -d $O/pmc_mem_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/pmc4_$TAG.log 2>&1 || { echo PMC4 FAILED; tail -5 $O/pmc4_$TAG.log; exit 1; }
echo MEASURE DONE
