# r05i: the measurement pass at the tree -- -m gpu suite, smoke, bench (with
# the CPU baseline), rocprofv3 kernel stats of both Atlas workloads, the mesh
# Atlas's fp64 MFMA and traffic PMC passes, the headline's traffic passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05i}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];r=d['roofline'];print('value',d['value'],d['kernels_ms'],r['frac'],r.get('frac_with_solvers'),'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'],'| cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'])"
B="python bench.py --no-cpu-baseline --no-mesh"
M="python bench.py --workload atlas_mesh --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- $B --steps 20 --warmup 3 > $O/prof_$T.log 2>&1 || { echo PROF FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mesh_$T -o run --output-format csv -- $M --steps 10 --warmup 2 > $O/prof_mesh_$T.log 2>&1 || { echo MESH PROF FAILED; exit 1; }
echo PROF OK
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc1_$T.log 2>&1 || { echo PMC1 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc2_$T.log 2>&1 || { echo PMC2 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc6_$T.log 2>&1 || { echo PMC6 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc7_$T.log 2>&1 || { echo PMC7 FAILED; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_$T -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/pmc5_$T.log 2>&1 || { echo PMC5 FAILED; tail -5 $O/pmc5_$T.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_mesh_$T -o run --output-format csv -- $M --steps 3 --warmup 1 > $O/pmc8_$T.log 2>&1 || { echo PMC8 FAILED; tail -5 $O/pmc8_$T.log; exit 1; }
echo PMC OK
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 120 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE2 FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
echo R05I DONE
