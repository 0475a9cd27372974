# A/B of library variants (dbg/libv*.so) on the two Atlas benches, no tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-var}
mkdir -p $O
for v in ${VARIANTS:-0 1 2 3 4}; do
  if [ "$v" = 0 ]; then LIB=$PWD/nimblephysics_amd/libnimble_amd.so; else LIB=$PWD/dbg/libv$v.so; fi
  NIMBLE_AMD_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/${T}_v$v.json 2> $O/${T}_v$v.err || { echo BENCH $v FAILED; tail -5 $O/${T}_v$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_v$v.json'));m=d['atlas_mesh'];print('v$v',round(d['value']),d['kernels_ms'],'| mesh',round(m['value']),m['kernels_ms']['forward'])"
done
echo VAR DONE
