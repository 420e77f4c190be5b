"""Run the native C++ host driver (csrc/host/mh_driver.cpp) on the bench
workload (gait10dof18musc, N=200, forward FD) at the bench iterate: the
IPOPT-iteration rate on host buffers (PCIe-inclusive: eval_f, eval_grad_f,
eval_g, eval_jac_g with g / J copied to the host) and the device-pointer
eval_g + eval_jac_g rate without Python in the loop.
usage: python tools/driver_bench.py [N] [steps] [keep_dir]
(keep_dir: write the tape and iterate there, kept, e.g. to profile the
driver binary itself under rocprofv3)"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))


def main():
    from mocohip import abi, configs
    from mocohip.tape import write_tape
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    steps = sys.argv[2] if len(sys.argv) > 2 else "200"
    st = configs.gait10dof18musc(N, fd_scheme="forward")
    rep = st.problem.create_rep()
    # the bench iterate (bounds midpoint states, random controls, seed 0)
    # computed with the oracle's identical bounds logic (no GPU context here)
    from mocohip.solver import OracleNLP
    ref = OracleNLP(rep, st.solver.options())
    x = ref.random_iterate(np.random.default_rng(0).uniform(-1, 1, ref.n))
    xm = ref.initial_guess_from_bounds()
    x[2:2 + ref.NS * ref.G] = xm[2:2 + ref.NS * ref.G]
    keep = sys.argv[3] if len(sys.argv) > 3 else None
    with tempfile.TemporaryDirectory() as d:
        if keep:
            os.makedirs(keep, exist_ok=True)
            d = keep
        tape, xf = os.path.join(d, "p.tape"), os.path.join(d, "x.bin")
        write_tape(rep, st.solver.options(), tape)
        x.tofile(xf)
        drv = os.path.join(ROOT, "opensim-moco_amd", "csrc", "build", "mh_driver")
        r = subprocess.run([drv, tape, "--steps", steps, "--x", xf], capture_output=True, text=True)
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)


if __name__ == "__main__":
    main()
