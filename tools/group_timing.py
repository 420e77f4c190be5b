"""k_groups critical path, group by group (timing diagnostic): the bench
workload (gait N=200 forward, generated rigid back end) with only group G's
blocks launched (MOCOHIP_DEBUG_GROUP, read at mh_create; results invalid),
DAE-stage device time per eval_jac_g from mh_debug_time_stages.
usage: python tools/group_timing.py [N] [G ...]
       python tools/group_timing.py rajagopal80 [N] [G ...]   (configs[3])"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))


def main():
    import torch
    from mocohip import configs
    from mocohip.solver import HipNLP
    args = sys.argv[1:]
    raja = bool(args) and args[0] == "rajagopal80"
    if raja:
        args = args[1:]
    N = int(args[0]) if args else 200
    groups = [int(a) for a in args[1:]] or [-1, 0, 1, 2, 4, 22, 27, 39]
    st = configs.rajagopal80(N, fd_scheme="forward") if raja else configs.gait10dof18musc(N, fd_scheme="forward")
    rep = st.problem.create_rep()
    for g in groups:
        os.environ["MOCOHIP_DEBUG_GROUP"] = str(g)
        nlp = HipNLP(rep, st.solver.options())
        x = nlp.random_iterate(np.random.default_rng(0).uniform(-1, 1, nlp.n))
        xm = nlp.initial_guess_from_bounds()
        x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
        xd = torch.tensor(x, dtype=torch.float64, device="cuda")
        dae, tr = nlp.time_stages(xd.data_ptr(), kind=1, reps=100)
        print(f"group {g:3d}: k_groups {1e3 * dae:7.2f} us  (transcription {1e3 * tr:7.2f} us)", flush=True)
        nlp.close()
    os.environ.pop("MOCOHIP_DEBUG_GROUP", None)


if __name__ == "__main__":
    main()
