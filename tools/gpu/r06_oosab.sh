#!/bin/bash
# OOS lines only (configs[3] incl. the measured full run and floor), default options and with elb_spec=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
A="--no-cpu --steps 2 --warmup 1 --bh-steps 0 --hy-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst --oos-chains 1"
timeout -k 10 400 python -u bench.py $A > gpurun_out/r06_oos_default.json 2> gpurun_out/r06_oos_default.err &&
timeout -k 10 400 python -u bench.py $A --opt elb_spec=1 > gpurun_out/r06_oos_spec.json 2> gpurun_out/r06_oos_spec.err
