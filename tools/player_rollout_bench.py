"""The per-player device rollout legs of bench.py alone (bench.secondary_player_rollout) as one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == '__main__':
    print(json.dumps(bench.secondary_player_rollout(torch.device('cuda', 0))))
