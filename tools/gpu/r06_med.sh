#!/bin/bash
# medium-ub truncated draw: the whole GPU suite, the floor probe, the bench without CPU lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06m}
timeout -k 10 800 python -u -m pytest -q -x -m gpu --timeout 240 --timeout-method thread tests/ > gpurun_out/full_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/full_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
