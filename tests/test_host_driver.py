"""The native C++ host (opensim-moco_amd/csrc/host/mh_driver.cpp) over the C
ABI: reads a problem tape written by mocohip.tape and drives the NLP
callbacks the way IPOPT's TNLP does."""
import os
import subprocess

import numpy as np
import pytest

from mocohip import configs
from mocohip.model import CoordinateCouplerConstraint, Function
from mocohip.tape import write_tape

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "opensim-moco_amd", "csrc", "build", "mh_driver")


def _run(*args):
    return subprocess.run([DRIVER, *map(str, args)], capture_output=True, text=True, timeout=120)


def test_driver_rejects_malformed_tape(tmp_path):
    bad = tmp_path / "bad.tape"
    bad.write_bytes(b"MHTAPE01" + b"\x01\x00\x00\x00" + b"\x00" * 10)
    r = _run(bad)
    assert r.returncode == 1 and "tape" in r.stderr


def test_driver_loads_tape_and_fails_loudly_without_gpu(tmp_path):
    """The tape parses completely (a truncated one is rejected before any
    HIP call); on a host without a gfx950 device mh_create reports it."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    st = configs.gait10dof18musc(4, control_bounds=True)
    # with a kinematic constraint: the tape carries it (version 4)
    st.problem.model.add_constraint(CoordinateCouplerConstraint(
        "knee_coupler", "knee_angle_l", Function.linear("knee_angle_r", 1.0, 0.0)))
    path = tmp_path / "gait.tape"
    write_tape(st.problem.create_rep(), st.solver.options(), str(path))
    r = _run(path)
    assert r.returncode == 2 and "no CPU fallback" in r.stderr, r.stderr
    # version 5: wraps (the Rajagopal model with its PathWraps kept)
    st5 = configs.rajagopal18_inverse(2, keep_path_wraps=True)
    p5 = tmp_path / "raja.tape"
    write_tape(st5.problem.create_rep(), st5.solver.options(), str(p5))
    r = _run(p5)
    assert r.returncode == 2 and "no CPU fallback" in r.stderr, r.stderr
    data = path.read_bytes()
    (tmp_path / "cut.tape").write_bytes(data[:-8])
    r = _run(tmp_path / "cut.tape")
    assert r.returncode == 1 and "malformed" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,mk", [
    ("gait_rigid", lambda: configs.gait10dof18musc(20)),
    ("double_pendulum_implicit", lambda: configs.double_pendulum(20, dynamics="implicit")),
    ("gait_pathcon", lambda: configs.gait10dof18musc(10, control_bounds=True)),
    ("coupled_pendulum", lambda: configs.double_pendulum_coupled(12, coupler="spline")),
    # tape v5: wrap surfaces / PathWraps; prescribed kinematics with coupler
    # multipliers, endpoint rows and detected sparsity
    ("wrapped_pendulum", lambda: configs.wrapped_pendulum(12, quadrant="-y")),
    ("rajagopal18_inverse_wrapped", lambda: configs.rajagopal18_inverse(3, keep_path_wraps=True)),
])
def test_driver_matches_python_binding_bit_exact(tmp_path, name, mk):
    """The C++ host and the ctypes binding drive the same library: same g and
    Jacobian values bit for bit at the same iterate."""
    import json
    from mocohip.solver import HipNLP
    st = mk()
    rep = st.problem.create_rep()
    nlp = HipNLP(rep, st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(4).uniform(-1, 1, nlp.n))
    xm = nlp.initial_guess_from_bounds()
    x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
    tape, xfile, out = tmp_path / "p.tape", tmp_path / "x.bin", tmp_path / "gj.bin"
    write_tape(rep, st.solver.options(), str(tape))
    x.tofile(xfile)
    r = _run(tape, "--steps", 5, "--warmup", 1, "--x", xfile, "--out", out)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n"] == nlp.n and line["nnz"] == nlp.nnz
    gj = np.fromfile(out)
    assert np.array_equal(gj[:nlp.m], nlp.eval_g(x))
    assert np.array_equal(gj[nlp.m:], nlp.eval_jac_g(x))
    assert line["f"] == nlp.eval_f(x)
