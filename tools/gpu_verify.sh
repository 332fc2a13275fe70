#!/bin/bash
# GPU-box check of the whole tree: parity tests, smoke, scan sweep, bench (logs under gpurun_out/).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=${1:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gputests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 200 python -u tools/scan_sweep.py > gpurun_out/${tag}_sweep.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1
