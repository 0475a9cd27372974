# final pass at HEAD: -m gpu suite, smoke, bench (with the CPU baseline), kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r04f}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];print('value',d['value'],d['kernels_ms'],d['roofline']['frac'],d['roofline']['traffic'],'| mesh',m['value'],m['kernels_ms']['forward'],m['traffic'],'| cpu',d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python bench.py --no-cpu-baseline --no-mesh --steps 20 --warmup 3 > $O/prof_$T.log 2>&1 || { echo PROF FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mesh_$T -o run --output-format csv -- python bench.py --workload atlas_mesh --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_mesh_$T.log 2>&1 || { echo MESH PROF FAILED; exit 1; }
echo FINAL DONE
