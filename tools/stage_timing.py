"""Per-call stage timing of the bench workload on the GPU: for eval_g,
eval_jac_g and the fused call, the host wall time per call and the HIP-event
stage times (mh_last_timings: whole, DAE stage, transcription stage).
Variants (env read at mh_create): default (k_interval), MOCOHIP_INTERVAL=0
(split k_combine + k_transcribe).
usage: python tools/stage_timing.py [N ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))


def main():
    import torch
    from mocohip import configs
    from mocohip.solver import HipNLP
    Ns = [int(a) for a in sys.argv[1:]] or [200, 400]
    variants = [{}, {"MOCOHIP_GRAPHS": "1"}, {"MOCOHIP_SPIN": "1"}, {"MOCOHIP_GRAPHS": "1", "MOCOHIP_SPIN": "1"}]
    for N, var in [(N, v) for N in Ns for v in variants]:
        for k in ("MOCOHIP_ORDER", "MOCOHIP_INTERVAL", "MOCOHIP_ASM", "MOCOHIP_QUOT", "MOCOHIP_EVENTS", "MOCOHIP_TABLES", "MOCOHIP_GRAPHS", "MOCOHIP_SPIN"):
            os.environ.pop(k, None)
        os.environ.update(var)
        st = configs.gait10dof18musc(N, fd_scheme="forward")
        rep = st.problem.create_rep()
        nlp = HipNLP(rep, st.solver.options())
        nlp.set_timing(True)
        x = nlp.random_iterate(np.random.default_rng(0).uniform(-1, 1, nlp.n))
        xm = nlp.initial_guess_from_bounds()
        x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
        xd = torch.tensor(x, dtype=torch.float64, device="cuda")
        gd = torch.zeros(nlp.m, dtype=torch.float64, device="cuda")
        vd = torch.zeros(nlp.nnz, dtype=torch.float64, device="cuda")
        calls = {
            "eval_g": lambda: nlp.eval_g_device(xd.data_ptr(), gd.data_ptr()),
            "eval_jac_g": lambda: nlp.eval_jac_g_device(xd.data_ptr(), vd.data_ptr()),
            "fused": lambda: nlp.eval_g_jac_g_device(xd.data_ptr(), gd.data_ptr(), vd.data_ptr()),
        }
        print(f"N={N} {var or 'default'} backend={nlp.backend()[0]} work={nlp.work()}")
        for name, fn in calls.items():
            for _ in range(5):
                fn()
            nlp.set_timing(False)
            W0 = []
            for _ in range(50):
                t0 = time.perf_counter()
                fn()
                W0.append(time.perf_counter() - t0)
            nlp.set_timing(True)
            T, W = [], []
            for _ in range(50):
                t0 = time.perf_counter()
                fn()
                W.append(time.perf_counter() - t0)
                T.append(nlp.last_timings())
            T = np.array(T)
            print(f"  {name:10s} wall {1e6 * np.median(W0):6.1f} us (timed {1e6 * np.median(W):6.1f})  events whole {1e3 * np.median(T[:, 0]):7.1f}"
                  f"  dae {1e3 * np.median(T[:, 1]):7.1f}  transcribe {1e3 * np.median(T[:, 2]):7.1f} us")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
