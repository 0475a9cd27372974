# one GPU pass at the current tree: -m gpu suite, smoke, bench (with the CPU
# baseline); TAG names the outputs under gpurun_out/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];r=d['roofline'];print('value',d['value'],d['kernels_ms'],r['frac'],r.get('frac_with_solvers'),r['traffic'],'| mesh',m['value'],m['kernels_ms']['forward'],m.get('frac_with_solvers'),'| cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'])"
echo PASS DONE
