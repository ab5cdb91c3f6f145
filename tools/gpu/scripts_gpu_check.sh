#!/bin/bash
# GPU round script: parity tests, smoke, rocprofv3 kernel stats, PMC passes
# (HBM bytes), then the bench (which reads the PMC summary).
# Every GPU step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01_v5}
: > gpurun_out/steps.log
step() { echo "== $1 $(date +%T)" >> gpurun_out/steps.log; }
if [ -z "$SKIP_TESTS" ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || exit 2
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
fi
step prof
rm -rf gpurun_out/prof gpurun_out/pmc_*
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || exit 5
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -s KILL 180 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_$c" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-profile > gpurun_out/pmc_$c.log 2>&1 || exit 6
done
mkdir -p profiles
python tools/pmc_summary.py profiles/${TAG}_pmc.json gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_summary.log 2>&1 || exit 7
cp profiles/${TAG}_pmc.json gpurun_out/
step bench
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 4
step done
