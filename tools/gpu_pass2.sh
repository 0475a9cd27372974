# one GPU pass at the tree: -m gpu suite, smoke, bench (CPU baseline on),
# rocprofv3 kernel stats of both Atlas workloads, the stage timing of both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05n}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];r=d['roofline'];c=d.get('cpu_baseline') or {};print('value',d['value'],d['kernels_ms'],r['frac'],r.get('frac_with_solvers'),'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'],'| cpu',c.get('value'),c.get('cores'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python bench.py --no-cpu-baseline --no-mesh --steps 20 --warmup 3 > $O/prof_$T.log 2>&1 || { echo PROF FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mesh_$T -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_mesh_$T.log 2>&1 || { echo MESH PROF FAILED; exit 1; }
grep -h -E "nimble_" $O/prof_$T/run_kernel_stats.csv $O/prof_mesh_$T/run_kernel_stats.csv | cut -d, -f1-4,6,7
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 120 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE2 FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
echo PASS DONE
