"""Per-block timing of k_groups (diagnostic build, `make -C
opensim-moco_amd/csrc task-timing`): for the bench workload prints, per
group, the block latency (shader cycles) and when its blocks started/ended
relative to the first block (wall clock, 100 MHz ticks -> us)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))


def main():
    import torch
    from mocohip import abi, configs
    from mocohip.solver import HipNLP
    path = os.path.join(ROOT, "opensim-moco_amd", "csrc", "build", "libmocohip_timing.so")
    lib = abi.load_mocohip(path)
    lib.mh_debug_task_timing.restype = C.c_int
    lib.mh_debug_task_timing.argtypes = [C.POINTER(C.c_longlong), C.c_int]
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    st = configs.gait10dof18musc(N, fd_scheme="forward")
    rep = st.problem.create_rep()
    nlp = HipNLP(rep, st.solver.options(), lib=lib)
    x = nlp.random_iterate(np.random.default_rng(0).uniform(-1, 1, nlp.n))
    xm = nlp.initial_guess_from_bounds()
    x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
    xd = torch.tensor(x, dtype=torch.float64, device="cuda")
    vd = torch.zeros(nlp.nnz, dtype=torch.float64, device="cuda")
    for _ in range(3):
        nlp.eval_jac_g_device(xd.data_ptr(), vd.data_ptr())
    print("timings ms", nlp.last_timings(), "work", nlp.work())
    ns = 1 << 16
    buf = (C.c_longlong * (5 * ns))()
    assert lib.mh_debug_task_timing(buf, ns) == 0
    a = np.frombuffer(buf, dtype=np.int64).reshape(ns, 5)
    a = a[a[:, 1] != 0]
    t0 = a[:, 1].min()
    print(f"{len(a)} blocks, span {(a[:, 2].max() - t0) / 100:.2f} us")
    lib.mh_debug_interval_timing.restype = C.c_int
    lib.mh_debug_interval_timing.argtypes = [C.POINTER(C.c_longlong), C.c_int]
    nb = 4096
    ib = (C.c_longlong * (4 * nb))()
    assert lib.mh_debug_interval_timing(ib, nb) == 0
    iv = np.frombuffer(ib, dtype=np.int64).reshape(nb, 4)
    iv = iv[iv[:, 0] != 0]
    if len(iv):
        z = iv[:, 0].min()
        d = np.diff(iv, axis=1) / 100.0
        print(f"k_interval: {len(iv)} blocks, span {(iv[:, 3].max() - z) / 100:.2f} us; start spread "
              f"{(iv[:, 0].max() - z) / 100:.2f} us; phase medians (us) stage {np.median(d[:, 0]):.2f} "
              f"combine {np.median(d[:, 1]):.2f} assemble {np.median(d[:, 2]):.2f}; max "
              f"{d[:, 0].max():.2f} {d[:, 1].max():.2f} {d[:, 2].max():.2f}")
    for g in np.unique(a[:, 0]):
        b = a[a[:, 0] == g]
        lat = b[:, 4] - b[:, 3]
        print(f"  group {g:3d}: {len(b):5d} blocks  cycles med {np.median(lat):7.0f} max {lat.max():7.0f}"
              f"  start us [{(b[:, 1].min() - t0) / 100:6.2f}, {(b[:, 1].max() - t0) / 100:6.2f}]"
              f"  end us max {(b[:, 2].max() - t0) / 100:6.2f}")


if __name__ == "__main__":
    main()
