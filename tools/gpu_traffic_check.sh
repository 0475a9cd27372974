set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=r04y
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests_$T.log; exit 1; }
tail -1 $O/gpu_tests_$T.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err || { echo BENCH FAILED; tail -5 $O/bench_$T.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_$T.json'));m=d['atlas_mesh'];print('value',d['value'],d['kernels_ms'],'| mesh',m['value'],m['kernels_ms']['forward'])"
B="python bench.py --no-cpu-baseline --no-mesh"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc1_$T.log 2>&1 || { echo PMC1 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc2_$T.log 2>&1 || { echo PMC2 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_mesh_$T -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc6_$T.log 2>&1 || { echo PMC6 FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_mesh_$T -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc7_$T.log 2>&1 || { echo PMC7 FAILED; exit 1; }
echo DONE
