"""The native C++ problem builder (opensim-moco_amd/csrc/host/mh_builder:
compileProblemRep's lowering in C++ -- Y order, default bounds rules,
goals / endpoint / path equations, frames, functions, muscles, wraps,
constraints, tables) against the Python lowering (mocohip/model.py,
mocohip/problem.py): the same study, described at the OpenSim level
(mocohip/describe.py) and built by the C++ tool, gives a problem tape
byte-identical to the one written from the Python ProblemRep -- so the
g / Jacobian the C ABI computes from it are the same bit for bit (checked on
the GPU through mh_driver below)."""
import os
import subprocess

import numpy as np
import pytest

from mocohip import configs
from mocohip.describe import write_description
from mocohip.problem import Constant, GCVSpline, MocoControlBoundConstraint, PiecewiseLinearFunction
from mocohip.tape import write_tape

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "opensim-moco_amd", "csrc", "build")
MH_BUILD = os.path.join(BUILD, "mh_build")


def _build(desc, tape, *extra):
    assert os.path.exists(MH_BUILD), "mh_build missing: run __graft_entry__.build()"
    return subprocess.run([MH_BUILD, str(desc), str(tape), *map(str, extra)], capture_output=True, text=True,
                          timeout=120)


def _bounded_pendulum(kind):
    st = configs.double_pendulum(12)
    pc = MocoControlBoundConstraint()
    pc.add_control_path("/tau0")
    pc.add_control_path("/tau1")
    if kind == "const":
        pc.set_lower_bound(Constant(-5.0))
        pc.set_upper_bound(Constant(7.5))
    elif kind == "pwl":
        pc.set_lower_bound(PiecewiseLinearFunction([0.0, 0.3, 0.71, 2.0], [-1.0, -2.5, 0.25, 1.0]))
    else:
        x = np.linspace(-0.1, 5.5, 9)
        pc.set_lower_bound(GCVSpline(5, x, np.sin(3 * x)))
        pc.set_equality_with_lower(True)
    st.problem.add_path_constraint(pc)
    return st


STUDIES = {
    "sliding_mass": lambda: configs.sliding_mass(7),
    "double_pendulum_swingup": lambda: configs.double_pendulum_swingup(9),
    "double_pendulum_implicit": lambda: configs.double_pendulum(8, dynamics="implicit"),
    "gait10dof18musc": lambda: configs.gait10dof18musc(6),
    "gait10dof18musc_compliant_central": lambda: configs.gait10dof18musc(5, tendon_compliance=True,
                                                                         fd_scheme="central"),
    "gait10dof18musc_pathcon": lambda: configs.gait10dof18musc(4, control_bounds=True),
    "gait10dof18musc_track": lambda: configs.gait10dof18musc_track(7),
    "gait10dof18musc_inverse": lambda: configs.gait10dof18musc_inverse(5),
    "rajagopal18_inverse_wrapped": lambda: configs.rajagopal18_inverse(3, keep_path_wraps=True),
    "rajagopal80_wrapped": lambda: configs.rajagopal80(3, keep_path_wraps=True),
    "coupled_pendulum_spline": lambda: configs.double_pendulum_coupled(6, coupler="spline"),
    "wrapped_pendulum_neg_y": lambda: configs.wrapped_pendulum(5, quadrant="-y"),
    "pendulum_bound_const": lambda: _bounded_pendulum("const"),
    "pendulum_bound_pwl": lambda: _bounded_pendulum("pwl"),
    "pendulum_bound_spline_eq": lambda: _bounded_pendulum("spline"),
    "pendulum_control_bound_both_implicit": lambda: configs.pendulum_control_bound(6, "both",
                                                                                   dynamics="implicit"),
    # tape v8: MocoParameters on a body mass / two springs' stiffness
    "oscillator_mass": lambda: configs.oscillator_mass(6),
    "oscillator_two_springs": lambda: configs.oscillator_two_springs(6),
}


@pytest.mark.parametrize("name", list(STUDIES))
def test_cpp_builder_tape_byte_identical(tmp_path, name):
    st = STUDIES[name]()
    desc, py_tape, cpp_tape = tmp_path / "s.mhdesc", tmp_path / "py.tape", tmp_path / "cpp.tape"
    write_description(st, str(desc))
    write_tape(st.problem.create_rep(), st.solver.options(), str(py_tape))
    r = _build(desc, cpp_tape)
    assert r.returncode == 0, r.stderr
    a, b = py_tape.read_bytes(), cpp_tape.read_bytes()
    assert len(a) == len(b)
    if a != b:
        first = next(i for i in range(len(a)) if a[i] != b[i])
        pytest.fail(f"tapes differ first at byte {first} of {len(a)}")


def test_cpp_builder_shard_options(tmp_path):
    st = configs.gait10dof18musc(8)
    desc, py_tape, cpp_tape = tmp_path / "s.mhdesc", tmp_path / "py.tape", tmp_path / "cpp.tape"
    write_description(st, str(desc))
    write_tape(st.problem.create_rep(), st.solver.options(3, 6), str(py_tape))
    r = _build(desc, cpp_tape, "--shard", 3, 6)
    assert r.returncode == 0, r.stderr
    assert py_tape.read_bytes() == cpp_tape.read_bytes()


def test_cpp_builder_reports_the_reference_errors(tmp_path):
    """The reference's input checks (MocoControlBoundConstraint.cpp:38-118,
    MocoControlGoal exponent) raise in the C++ builder too."""
    cases = []
    st = configs.double_pendulum(4)
    pc = MocoControlBoundConstraint()
    pc.add_control_path("/tau0")
    pc.set_lower_bound(Constant(1.0))
    pc.set_upper_bound(Constant(2.0))
    pc.set_equality_with_lower(True)
    st.problem.add_path_constraint(pc)
    cases.append((st, "upper bound function must not be set"))
    st = configs.double_pendulum(4)
    pc = MocoControlBoundConstraint()
    pc.add_control_path("/tau0")
    x = np.linspace(0.5, 0.9, 6)
    pc.set_lower_bound(GCVSpline(5, x, x))
    st.problem.add_path_constraint(pc)
    cases.append((st, "minimum domain value"))
    st = configs.double_pendulum(4)
    next(g for g in st.problem.goals if hasattr(g, "control_weights")).exponent = 1
    cases.append((st, "Exponent must be 2 or greater"))
    st = configs.oscillator_mass(4)
    st.problem.parameters[0].property_name = "mass_center"
    cases.append((st, "needs an element in [0, 3)"))
    st = configs.oscillator_two_springs(4)
    st.problem.parameters[0].component_paths.append("/forceset/nosuchspring")
    cases.append((st, "no component '/forceset/nosuchspring'"))
    st = configs.oscillator_mass(4)
    st.problem.parameters[0].property_name = "stiffness"
    cases.append((st, "has no property 'stiffness'"))
    for i, (st, msg) in enumerate(cases):
        desc = tmp_path / f"e{i}.mhdesc"
        write_description(st, str(desc))
        r = _build(desc, tmp_path / f"e{i}.tape")
        assert r.returncode == 1 and msg in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gait10dof18musc", "rajagopal18_inverse_wrapped", "pendulum_bound_pwl",
                                  "oscillator_two_springs"])
def test_cpp_built_tape_drives_the_library_like_python(tmp_path, name):
    """g and the Jacobian values the C ABI computes from the C++-built tape
    (mh_driver) equal the Python binding's on the Python-lowered problem."""
    import json
    from mocohip.solver import HipNLP
    st = STUDIES[name]()
    rep = st.problem.create_rep()
    nlp = HipNLP(rep, st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(6).uniform(-1, 1, nlp.n))
    x[2:2 + nlp.NS * nlp.G] = nlp.initial_guess_from_bounds()[2:2 + nlp.NS * nlp.G]
    desc, tape, xfile, out = (tmp_path / "s.mhdesc", tmp_path / "cpp.tape", tmp_path / "x.bin",
                              tmp_path / "gj.bin")
    write_description(st, str(desc))
    assert _build(desc, tape).returncode == 0
    x.tofile(xfile)
    r = subprocess.run([os.path.join(BUILD, "mh_driver"), str(tape), "--steps", "3", "--warmup", "1",
                        "--x", str(xfile), "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n"] == nlp.n and line["nnz"] == nlp.nnz
    gj = np.fromfile(out)
    assert np.array_equal(gj[:nlp.m], nlp.eval_g(x))
    assert np.array_equal(gj[nlp.m:], nlp.eval_jac_g(x))
    nlp.close()
