"""A/B of the host entries' chunked Jacobian copy (MOCOHIP_D2H_CHUNKS, read
at mh_create): eval_g + eval_jac_g on page-locked host buffers, calls/s, for
1 (one copy after the assembly) and 2 / 4 / 8 chunks, gait N=200 and 400.
usage: python tools/d2h_chunks_ab.py [N ...]"""
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
    for N in Ns:
        st = configs.gait10dof18musc(N, fd_scheme="forward")
        rep = st.problem.create_rep()
        for ch in ("1", "2", "4", "8"):
            os.environ["MOCOHIP_D2H_CHUNKS"] = ch
            nlp = HipNLP(rep, st.solver.options())
            x = nlp.random_iterate(np.random.default_rng(0).uniform(-1, 1, nlp.n))
            x[2:2 + nlp.NS * nlp.G] = nlp.initial_guess_from_bounds()[2:2 + nlp.NS * nlp.G]
            xh = torch.tensor(x).pin_memory().numpy()
            g = torch.zeros(nlp.m, dtype=torch.float64).pin_memory().numpy()
            v = torch.zeros(nlp.nnz, dtype=torch.float64).pin_memory().numpy()
            import ctypes as C
            from mocohip import abi
            for _ in range(20):
                nlp.lib.mh_eval_g(nlp.ctx, abi.dptr(xh), 1, abi.dptr(g))
                nlp.lib.mh_eval_jac_g(nlp.ctx, abi.dptr(xh), 0, abi.dptr(v))
            k = 200
            t0 = time.perf_counter()
            for _ in range(k):
                nlp.lib.mh_eval_g(nlp.ctx, abi.dptr(xh), 1, abi.dptr(g))
                nlp.lib.mh_eval_jac_g(nlp.ctx, abi.dptr(xh), 0, abi.dptr(v))
            el = time.perf_counter() - t0
            t0 = time.perf_counter()
            for _ in range(k):
                nlp.lib.mh_eval_g_jac_g(nlp.ctx, abi.dptr(xh), abi.dptr(g), abi.dptr(v))
            elf = time.perf_counter() - t0
            print(f"N={N} chunks={ch}: separate {k / el:8.1f} calls/s ({1e3 * el / k:.3f} ms), "
                  f"fused {k / elf:8.1f} calls/s ({1e3 * elf / k:.3f} ms), J {8 * nlp.nnz / 1e6:.1f} MB",
                  flush=True)
            nlp.close()
    os.environ.pop("MOCOHIP_D2H_CHUNKS", None)


if __name__ == "__main__":
    main()
