"""Geister learner step (B=256 T=16, HIP graph) with the deferred convs' input gradient on aten (MIOpen) vs
hrl_gboard's adjoint conv (nn.GBOARD_ADJOINT), and the recurrent learner's losses against the CPU oracle.

    python tools/adjoint_bench.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if len(sys.argv) > 1:
        sys.path.insert(0, ROOT)
        from handyrl_amd import nn as hnn
        hnn.GBOARD_ADJOINT = sys.argv[1] == '1'
        sys.argv = [sys.argv[0], '--B', '256', '--T', '16', '--graph', '1']
        import runpy
        runpy.run_path(os.path.join(ROOT, 'tools', 'geister_bench.py'), run_name='__main__')
        return
    for flag in ('0', '1', '0', '1'):
        out = subprocess.run([sys.executable, os.path.abspath(__file__), flag], capture_output=True, text=True)
        lines = [l for l in out.stdout.splitlines() if l.startswith('{')]
        print(json.dumps({'gboard_adjoint': flag == '1', 'result': json.loads(lines[-1]) if lines else out.stderr[-400:]}),
              flush=True)


if __name__ == '__main__':
    main()
