#!/bin/bash
# r06i: -m gpu suite, smoke, bench, and the headline forward's HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06i}
mkdir -p $O
bash tools/gpu_r06.sh skip-wide || exit 1
B="python bench.py --no-cpu-baseline --no-mesh"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc1_$T.log 2>&1 || { echo PMC1 FAILED; tail -5 $O/pmc1_$T.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_$T -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/pmc2_$T.log 2>&1 || { echo PMC2 FAILED; tail -5 $O/pmc2_$T.log; exit 1; }
python tools/pmc_traffic.py $O/pmc_fetch_$T $O/pmc_write_$T 1024 atlas $O/pmc_traffic_$T.json > /dev/null && python -c "import json;d=json.load(open('$O/pmc_traffic_$T.json'))['atlas'];print({k:(round(v['write_kib']),round(v['fetch_kib_raw']),round(v['bytes_per_world'])) for k,v in d.items()})"
echo R06I DONE
