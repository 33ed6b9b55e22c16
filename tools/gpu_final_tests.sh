#!/bin/bash
# The full -m gpu suite and smoke() on the tree's build, as the driver runs them.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05_gputests.log 2>&1 || { tail -40 gpurun_out/r05_gputests.log; exit 1; }
tail -3 gpurun_out/r05_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
