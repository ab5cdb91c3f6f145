#!/bin/bash
# bench.py default run (incl. the measured floor and full configs[3] run), then the A-step phase
# attribution at the floor (ablation build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05q}
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so timeout -k 10 120 python tools/dbg/astep_prof.py 5 \
  > gpurun_out/astep_prof_$TAG.json
