"""configs[4]: the batch of MocoInverse solves on one GPU (mocohip.batchsolve)
with a given linear solver; one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "opensim-moco_amd"))
from mocohip import batchsolve  # noqa: E402

if __name__ == "__main__":      # spawned workers re-import this file
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ls = sys.argv[2] if len(sys.argv) > 2 else "auto"
    out = batchsolve.solve_batch(batchsolve.sweep(B), 125, linear_solver=ls)
    print(json.dumps(out), flush=True)
