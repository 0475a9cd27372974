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
B="python bench.py --no-cpu-baseline --no-mesh $*"
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
# other workloads: the STL-mesh Atlas (the reference atlas_bench's model,
# LCPs up to 96 rows) and configs[1] cartpole, bench lines + kernel stats
timeout -k 10 300 python bench.py --workload atlas_mesh --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_atlas_mesh_$TAG.json 2> $O/bench_atlas_mesh_$TAG.err || { echo MESH BENCH FAILED; tail -20 $O/bench_atlas_mesh_$TAG.err; exit 1; }
cut -c1-1500 $O/bench_atlas_mesh_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mesh_$TAG -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_mesh_$TAG.log 2>&1 || { echo MESH PROF FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_mesh_$TAG -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc6_$TAG.log 2>&1 || { echo PMC6 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_mesh_$TAG -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc7_$TAG.log 2>&1 || { echo PMC7 FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cartpole_$TAG -o run --output-format csv -- python bench.py --workload cartpole --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_cartpole_$TAG.log 2>&1 || { echo CARTPOLE PROF FAILED; exit 1; }
timeout -k 10 120 python bench.py --workload cartpole --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_cartpole_$TAG.json 2>&1 || { echo CARTPOLE BENCH FAILED; exit 1; }
timeout -k 10 120 python bench.py --workload half_cheetah --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_half_cheetah_$TAG.json 2>&1 || { echo HALF CHEETAH BENCH FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_half_cheetah_$TAG -o run --output-format csv -- python bench.py --workload half_cheetah --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_half_cheetah_$TAG.log 2>&1 || { echo HALF CHEETAH PROF FAILED; exit 1; }
echo WORKLOADS OK
# fp64 matrix-core counters (last: a counter this rocprof does not know ends
# only this pass); summarised here by tools/pmc_mfma.py -> profiles/pmc_mfma.json
timeout -s KILL 60 rocprofv3 -L > $O/counters_$TAG.txt 2>&1
grep -i -E "MFMA|MOPS" $O/counters_$TAG.txt | head -20
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/pmc5_$TAG.log 2>&1 || { echo PMC5 FAILED; tail -5 $O/pmc5_$TAG.log; exit 1; }
echo MEASURE DONE
