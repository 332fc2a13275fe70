#!/bin/bash
# round 6: the per-player device rollout -- reference-game parity on the GPU (eager and graph), the main-entry
# device modes, the step-tail / gloo tests touched this round, then the per-player rollout bench legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6f
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rollout_players.py \
  "tests/test_main_entry.py::test_train_main_device_player_modes_gpu" tests/test_rollout.py > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 600 python3 tools/player_rollout_bench.py > $out/player_rollout.json 2> $out/player_rollout.err || { tail -20 $out/player_rollout.err; exit 1; }
cat $out/player_rollout.json
