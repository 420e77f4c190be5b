"""The plugin's trajectory conversion in C++ (opensim-moco_amd/csrc/host/
mh_trajectory.hpp: the MocoHipSolver plugin's toSolution / toIterate,
integration/MocoHipSolver.cpp; driven here through ``mh_build --solution``)
carries EVERY variable block by the reference's names -- states, controls,
multipliers (lambda_cid<c>_p0), derivatives (<coordinate>/accel,
<muscle>/implicitderiv_normalized_tendon_force), slacks (gamma_cid<c>_p0)
-- and parameters (MocoParameter names) as MocoCasOCProblem.h:70-187 converts CasOC iterates, and converts back
to the same iterate bit for bit.

Checked against the Python conversion (mocohip.trajectory.MocoTrajectory.
from_iterate) on the C++-built problem of the same study, and against the
reference's own MocoInverse solution file: its lambda / implicitderiv
columns come out of the C++ path under the file's own names with the file's
values (the golden solution's iterate), and a converged solve's columns are
within the file's tolerance of them (the solve through the oracle on the CPU
here; on the device in tests/test_solve.py)."""
import json
import os
import subprocess

import numpy as np
import pytest

from mocohip import configs
from mocohip.describe import write_description
from mocohip.solver import OracleNLP
from mocohip.trajectory import MocoTrajectory

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MH_BUILD = os.path.join(ROOT, "opensim-moco_amd", "csrc", "build", "mh_build")
GOLDEN = os.path.join(ROOT, "tests", "golden", "std_testMocoInverse_subject_18musc_solution.npz")


def _cpp_solution(tmp_path, st, x):
    """mh_build's .sto of iterate x (the C++ builder's rep of the study)."""
    desc, tape, xb, sto = (tmp_path / "s.mhdesc", tmp_path / "s.tape", tmp_path / "x.bin",
                           tmp_path / "sol.sto")
    write_description(st, str(desc))
    np.ascontiguousarray(x, np.float64).tofile(str(xb))
    r = subprocess.run([MH_BUILD, str(desc), str(tape), "--solution", str(xb), str(sto)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout)
    assert info["roundtrip"] is True, info
    return MocoTrajectory.read(str(sto)), info


STUDIES = {
    "rajagopal18_inverse": lambda: configs.rajagopal18_inverse(4, sparsity="none"),
    "coupled_pendulum": lambda: configs.double_pendulum_coupled(5),
    "coupled_pendulum_implicit": lambda: configs.double_pendulum_coupled(4, dynamics="implicit"),
    "gait_implicit_both": lambda: configs.gait10dof18musc(3, tendon_compliance=True, tendon_dynamics="implicit",
                                                          dynamics="implicit"),
    "gait_inverse": lambda: configs.gait10dof18musc_inverse(3, sparsity="none"),
    # MocoParameters: the last block, one value each (the .sto's first row)
    "oscillator_mass": lambda: configs.oscillator_mass(4),
    "gait_parameters_implicit": lambda: configs.gait10dof18musc_parameters(3, dynamics="implicit"),
}


@pytest.mark.parametrize("name", list(STUDIES))
def test_cpp_solution_matches_python_conversion(tmp_path, name):
    st = STUDIES[name]()
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(2).uniform(-1, 1, nlp.n))
    cpp, info = _cpp_solution(tmp_path, st, x)
    assert info["n"] == nlp.n
    py = MocoTrajectory.from_iterate(nlp, x)
    for b in ("state", "control", "multiplier", "derivative", "slack", "parameter"):
        assert getattr(cpp, b + "_names") == getattr(py, b + "_names"), b
        assert np.array_equal(getattr(cpp, b + "s"), getattr(py, b + "s"), equal_nan=True), b
    assert len(cpp.parameter_names) == nlp.NPAR
    assert np.array_equal(cpp.time, py.time)
    # every block named the reference's way
    if nlp.NM:
        assert all(n.startswith("lambda_cid") for n in cpp.multiplier_names)
    if nlp.NSL:
        assert [n.replace("gamma", "lambda") for n in cpp.slack_names] == cpp.multiplier_names
    if nlp.NDV:
        assert all(n.endswith("/accel") or "/implicitderiv_" in n for n in cpp.derivative_names)
    # and the Python conversion back gives the iterate (resampled at its own
    # grid times by the interpolating GCV spline: to rounding)
    assert np.allclose(py.to_iterate(nlp), x, rtol=1e-10, atol=1e-10)
    nlp.close()


def _golden():
    d = np.load(GOLDEN)
    return [str(s) for s in d["labels"]], d["data"]


def test_cpp_solution_golden_columns():
    """The reference's MocoInverse solution (Rajagopal 18, N = 11) as an
    iterate of our NLP, through the C++ conversion: the file's multiplier and
    implicit-derivative columns come back under the file's own names, value
    for value on the grid."""
    import tempfile
    from pathlib import Path
    st = configs.rajagopal18_inverse()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    labels, data = _golden()
    col = {l: i for i, l in enumerate(labels)}
    assert len(data) == nlp.G
    gold = MocoTrajectory(data[:, 0], list(rep.state_names), list(rep.control_names),
                          [l for l in labels if l.startswith("lambda")],
                          [l for l in labels if "implicitderiv" in l],
                          states=data[:, [col[n] for n in rep.state_names]],
                          controls=data[:, [col[n] for n in rep.control_names]],
                          multipliers=data[:, [col[l] for l in labels if l.startswith("lambda")]],
                          derivatives=data[:, [col[l] for l in labels if "implicitderiv" in l]])
    x = gold.to_iterate(nlp)
    with tempfile.TemporaryDirectory() as d:
        cpp, _ = _cpp_solution(Path(d), st, x)
    for names, block in ((cpp.multiplier_names, cpp.multipliers), (cpp.derivative_names, cpp.derivatives)):
        assert names and all(n in col for n in names), names
        for j, n in enumerate(names):
            ref = data[:, col[n]]
            assert np.allclose(block[:, j], ref, rtol=1e-9, atol=1e-9 * (1 + np.abs(ref).max())), n
    nlp.close()


def _blocks_rms(gold_labels, gold_data, traj):
    """(multipliers, derivatives, states, controls) RMS of ``traj`` against
    the golden file, MocoTrajectory::compareContinuousVariablesRMS per
    block."""
    col = {l: i for i, l in enumerate(gold_labels)}

    def sub(names):
        return gold_data[:, [col[n] for n in names]]
    gold = MocoTrajectory(gold_data[:, 0], list(traj.state_names), list(traj.control_names),
                          list(traj.multiplier_names), list(traj.derivative_names),
                          states=sub(traj.state_names), controls=sub(traj.control_names),
                          multipliers=sub(traj.multiplier_names), derivatives=sub(traj.derivative_names))
    none = ["none"]
    return (gold.compare_continuous_variables_rms(traj, states=none, controls=none, derivatives=none),
            gold.compare_continuous_variables_rms(traj, states=none, controls=none, multipliers=none),
            gold.compare_continuous_variables_rms(traj, controls=none, multipliers=none, derivatives=none),
            gold.compare_continuous_variables_rms(traj, states=none, multipliers=none, derivatives=none))


def test_cpp_solution_of_a_solve_against_golden(tmp_path):
    """testMocoInverse.cpp:118-147 solved (here through the oracle on the
    CPU, host linear algebra; the device solve: tests/test_solve.py), its
    iterate written as the plugin's MocoSolution by the C++ conversion: the
    states and controls within the reference's own 1e-2 RMS of
    std_testMocoInverse_subject_18musc_solution.sto (testMocoInverse.cpp:
    144-146), and the columns the reference does not assert -- the coupler
    multipliers and the tendon-force derivatives, weakly determined at the
    MocoInverse tolerance 1e-3 -- under the file's names within 2e-2 / 6e-2
    RMS of it (magnitudes up to 8.5 and 4.3; measured 0.012 / 0.031)."""
    st = configs.rajagopal18_inverse()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options(), threads=8)
    sol = st.solve(nlp=nlp, linear_solver="host")
    assert sol.metadata["success"] == "true"
    cpp, _ = _cpp_solution(tmp_path, st, sol.stats.x)
    labels, data = _golden()
    rm, rd, rs, rc = _blocks_rms(labels, data, cpp)
    print(f"RMS vs golden: multipliers {rm:.4f}, derivatives {rd:.4f}, states {rs:.4f}, controls {rc:.4f}")
    assert rs < 1e-2 and rc < 1e-2, (rs, rc)
    assert rm < 2e-2 and rd < 6e-2, (rm, rd)
    nlp.close()
