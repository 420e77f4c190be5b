"""Diagnostic: async eval_g_jac_g_device calls/s driven from Python, with
and without torch in the process (device buffers from hipMalloc via ctypes),
against the native driver's figure.  usage: python tools/py_overhead.py [torch]"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))


def main():
    use_torch = len(sys.argv) > 1 and sys.argv[1] == "torch"
    if use_torch:
        import torch
        torch.zeros(1, device="cuda")
    from mocohip import configs
    from mocohip.solver import HipNLP
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    st = configs.gait10dof18musc(200, fd_scheme="forward")
    nlp = HipNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.initial_guess_from_bounds()
    ptrs = []
    for n in (nlp.n, nlp.m, nlp.nnz):
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), 8 * n) == 0
        ptrs.append(p.value)
    assert hip.hipMemcpy(ptrs[0], x.ctypes.data, 8 * nlp.n, 1) == 0
    nlp.set_async(True)
    fn = nlp.lib.mh_eval_g_jac_g_device
    ctx = nlp.ctx
    xp, gp, vp = (C.c_void_p(p) for p in ptrs)
    for label, call in (("HipNLP.eval_g_jac_g_device", lambda: nlp.eval_g_jac_g_device(*ptrs)),
                        ("bare ctypes", lambda: fn(ctx, xp, gp, vp))):
        for _ in range(50):
            call()
        nlp.synchronize()
        K = 2000
        t = time.perf_counter()
        for _ in range(K):
            call()
        nlp.synchronize()
        el = time.perf_counter() - t
        print(f"torch={use_torch} {label}: {K / el:.0f} calls/s ({1e6 * el / K:.1f} us/call)", flush=True)


if __name__ == "__main__":
    main()
