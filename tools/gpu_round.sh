#!/bin/bash
# One GPU-box session: smoke, bench, rocprofv3 kernel trace (summary CSVs
# land in gpurun_out/prof_<tag>/).  Usage: bash tools/gpu_round.sh <tag> [bench args]
set -o pipefail
TAG=${1:-r01}
shift || true
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $R/gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py "$@" > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 $R/gpurun_out/bench_$TAG.err; exit 1; }
cat $R/gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*stats*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $R/gpurun_out/pmc1_$TAG.log 2>&1 || { echo PMC1 FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $R/gpurun_out/pmc2_$TAG.log 2>&1 || { echo PMC2 FAILED; exit 1; }
echo PMC OK
