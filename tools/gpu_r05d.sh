# r05d: tests, headline + mesh bench, mesh WRITE_SIZE, mesh stage timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05d}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -5 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];print('atlas',d['value'],d['kernels_ms'],'mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/${T}_pmc_write_mesh -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/${T}_pmc_w.log 2>&1 || { echo PMCW FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/${T}_pmc_fetch_mesh -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/${T}_pmc_f.log 2>&1 || { echo PMCF FAILED; exit 1; }
python tools/pmc_traffic.py $O/${T}_pmc_fetch_mesh $O/${T}_pmc_write_mesh 1024 atlas_mesh $O/${T}_pmc_traffic_mesh.json > /dev/null && python -c "import json;d=json.load(open('$O/${T}_pmc_traffic_mesh.json'))['atlas_mesh'];print({k:(round(v['bytes_per_world']),round(v['write_kib']*1024/v['launches']/1024)) for k,v in d.items()})"
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
echo R05D DONE
