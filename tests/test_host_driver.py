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
    # version 8: springs + MocoParameters
    st8 = configs.oscillator_two_springs(5)
    p8 = tmp_path / "osc.tape"
    write_tape(st8.problem.create_rep(), st8.solver.options(), str(p8))
    r = _run(p8)
    assert r.returncode == 2 and "no CPU fallback" in r.stderr, r.stderr
    data = path.read_bytes()
    (tmp_path / "cut.tape").write_bytes(data[:-8])
    r = _run(tmp_path / "cut.tape")
    assert r.returncode == 1 and "malformed" in r.stderr


def test_driver_checks_the_guess_size(tmp_path):
    """The initial-guess iterate on a tape (tape v8) is the whole x: n
    doubles (mh_options.sparsity_guess), sized with mh_get_nlp_info_for
    before any device call; the driver rejects a guess blob of another size,
    and the Python side refuses a guess array of the wrong size."""
    import ctypes as C
    import struct
    from mocohip import abi
    from mocohip.solver import check_guess_size
    st = configs.double_pendulum(5)
    rep = st.problem.create_rep()
    st.solver.optim_sparsity_detection = "initial-guess"
    info = abi.mh_nlp_info()
    opts = st.solver.options()
    assert abi.load_mocohip().mh_get_nlp_info_for(C.byref(rep.struct), C.byref(opts), C.byref(info)) == 0
    n = int(info.n)
    st.solver.sparsity_guess = np.linspace(-0.5, 0.5, n + 1)
    with pytest.raises(ValueError, match="sparsity_guess has"):
        check_guess_size(rep, st.solver.options())
    st.solver.sparsity_guess = np.linspace(-0.5, 0.5, n)
    opts = st.solver.options()
    check_guess_size(rep, opts)
    path = tmp_path / "g.tape"
    write_tape(rep, opts, str(path))
    data = path.read_bytes()
    key = struct.pack("<q", 8 * n) + np.linspace(-0.5, 0.5, n).tobytes()
    at = data.find(key)
    assert at > 0
    r = _run(path)
    assert "initial-guess iterate" not in r.stderr, r.stderr
    bad = data[:at] + struct.pack("<q", 8 * (n - 1)) + data[at + 8:at + 8 * n] + data[at + 8 + 8 * n:]
    (tmp_path / "bad.tape").write_bytes(bad)
    r = _run(tmp_path / "bad.tape")
    assert r.returncode == 1 and "initial-guess iterate has" in r.stderr, r.stderr


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
    # tape v8: springs and MocoParameters
    ("oscillator_two_springs", lambda: configs.oscillator_two_springs(12)),
    ("oscillator_mass", lambda: configs.oscillator_mass(12)),
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
