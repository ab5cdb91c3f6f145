#!/bin/bash
# kernel timeline of the OOS floor probe (rocprofv3 kernel trace), spec off / on
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sp in 0 1; do
  rm -rf gpurun_out/r06_trace_spec$sp
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06_trace_spec$sp" -o run --output-format csv -- \
    python "$R/tools/probe_floor.py" 6 elb_spec=$sp noprof > gpurun_out/r06_trace_spec$sp.log 2>&1 || exit 1
done
