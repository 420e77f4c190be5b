"""Quick GPU-vs-oracle diagnostic (prints max differences per config)."""
import sys, time, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))
from mocohip import configs
from mocohip.solver import HipNLP, OracleNLP

cases = [("sm", configs.sliding_mass(50)), ("dp", configs.double_pendulum(100)),
         ("dp_trap", configs.double_pendulum(50, "trapezoidal")),
         ("gait20", configs.gait10dof18musc(20)),
         ("gait20c", configs.gait10dof18musc(20, tendon_compliance=True, fd_scheme="central"))]
for name, st in cases:
    rep = st.problem.create_rep()
    opts = st.solver.options()
    t = time.time()
    gpu = HipNLP(rep, opts)
    ref = OracleNLP(rep, opts, threads=8)
    x = gpu.random_iterate(np.random.default_rng(0).uniform(-1, 1, gpu.n))
    x0 = gpu.initial_guess_from_bounds()
    for xx, lab in [(x, "rand"), (x0, "mid")]:
        ir, jc = gpu.jac_structure(); ir0, jc0 = ref.jac_structure()
        g, g0 = gpu.eval_g(xx), ref.eval_g(xx)
        J, J0 = gpu.eval_jac_g(xx), ref.eval_jac_g(xx)
        f, f0 = gpu.eval_f(xx), ref.eval_f(xx)
        gf, gf0 = gpu.eval_grad_f(xx), ref.eval_grad_f(xx)
        rel = lambda a, b: np.abs(a - b).max() / max(1e-300, np.abs(b).max())
        print(f"{name:8s} {lab}: struct_eq={np.array_equal(ir,ir0) and np.array_equal(jc,jc0)} "
              f"g rel={rel(g,g0):.2e} J rel={rel(J,J0):.2e} f={f:.6g}/{f0:.6g} gradf rel={rel(gf,gf0):.2e} "
              f"nanJ={np.isnan(J).sum()}", flush=True)
    # timing
    for _ in range(3): gpu.eval_jac_g(x)
    t = time.time(); n = 20
    for _ in range(n): gpu.eval_jac_g(x)
    dt = (time.time() - t) / n
    print(f"   jac_g {dt*1e3:.3f} ms/call (host), kernel timings {gpu.last_timings()}", flush=True)
