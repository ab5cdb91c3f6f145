#!/bin/bash
# k_phi with Z staged in LDS + X'v chain pairs in the split solve: tests, floor probe, phases, main line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06h}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mirror.py tests/test_gpu_lag.py tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/t_$TAG.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so timeout -k 10 200 python -u tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.err &&
timeout -k 10 300 python -u bench.py --no-cpu --bh-steps 0 --hy-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst --oos-steps 0 --oos-full-draws 0 > gpurun_out/main_$TAG.json 2> gpurun_out/main_$TAG.err
