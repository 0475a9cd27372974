# forward LDS pool rows (NIMBLE_AMD_LDS_ROWS) on the mesh Atlas: bench value per setting
set -o pipefail
for r in ${ROWS:-24 36 40 44 48}; do
  NIMBLE_AMD_VERBOSE=1 NIMBLE_AMD_LDS_ROWS=$r timeout -k 10 200 python bench.py --workload atlas_mesh --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/rows_$r.json 2> gpurun_out/rows_$r.err || { echo "rows $r FAILED"; tail -5 gpurun_out/rows_$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rows_$r.json'));print('rows $r', round(d['value']), d['kernels_ms'])"
  grep -h "LDS forward\|defers" gpurun_out/rows_$r.err | head -2
done
