#!/bin/bash
# r06 final measurement pass at HEAD: bench (with the CPU baseline),
# rocprofv3 kernel stats (headline, mesh Atlas, cartpole, half-cheetah),
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and fp64 MFMA PMC of
# the headline and the mesh Atlas, and the stage-timing histograms
# (-DNIMBLE_STAGE_TIMING build in dbg/).  Every GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06m}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-mesh"
M="python bench.py --workload atlas_mesh --no-cpu-baseline"
timeout -k 10 400 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];print('value',d['value'],d['kernels_ms'],d['roofline']['frac'],'| mesh',m['value'],m['kernels_ms']['forward'],'| cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- $B --steps 20 --warmup 3 > $O/prof_$T.log 2>&1 || { echo PROF FAILED; tail -5 $O/prof_$T.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mesh_$T -o run --output-format csv -- $M --steps 10 --warmup 3 > $O/prof_mesh_$T.log 2>&1 || { echo MESH PROF FAILED; tail -5 $O/prof_mesh_$T.log; exit 1; }
echo PROF OK
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc1_$T.log 2>&1 || { echo PMC1 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc2_$T.log 2>&1 || { echo PMC2 FAILED; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc3_$T.log 2>&1 || { echo PMC3 FAILED; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc4_$T.log 2>&1 || { echo PMC4 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_$T -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/pmc5_$T.log 2>&1 || { echo PMC5 FAILED; tail -5 $O/pmc5_$T.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc6_$T.log 2>&1 || { echo PMC6 FAILED; tail -5 $O/pmc6_$T.log; exit 1; }
echo PMC OK
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 200 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE MESH FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
echo STAGE OK
timeout -k 10 200 python bench.py --workload cartpole --no-cpu-baseline --steps 20 --warmup 3 > $O/${T}_bench_cartpole.json 2>/dev/null || { echo CARTPOLE FAILED; exit 1; }
timeout -k 10 200 python bench.py --workload half_cheetah --no-cpu-baseline --steps 20 --warmup 3 > $O/${T}_bench_half_cheetah.json 2>/dev/null || { echo CHEETAH FAILED; exit 1; }
echo MEASURE DONE
