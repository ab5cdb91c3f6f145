#!/bin/bash
# the whole GPU suite on the current tree
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
tail -3 $O/suite.log; exit $rc
