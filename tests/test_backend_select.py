"""Which device back end mh_create selects (mh_backend_for: host only, no
GPU): the generated model-specialized kernels are specialized on the model
STRUCTURE, so models that differ only in their numbers -- a heavier femur, a
scaled subject, another trial's data -- keep them;
structural changes fall back to the generic interpreter."""
import ctypes as C

import numpy as np
import pytest

from mocohip import abi, configs


def _backend(st):
    lib = abi.load_mocohip()
    rep = st.problem.create_rep()
    opts = st.solver.options()
    buf = C.create_string_buffer(128)
    rc = lib.mh_backend_for(C.byref(rep.struct), C.byref(opts), buf, 128)
    assert rc == 0, lib.mh_last_error()
    return buf.value.decode()


def test_bundled_models_select_their_generated_back_end():
    assert _backend(configs.gait10dof18musc(4)) == "generated:gait10dof18musc_rigid"
    assert _backend(configs.gait10dof18musc(4, muscles=False)) == "generated:gait10dof18musc_torque"
    assert _backend(configs.gait10dof18musc(4, dynamics="implicit")) == \
        "generated:gait10dof18musc_rigid_implicit"
    assert _backend(configs.gait10dof18musc_inverse(4)) == "generated:gait10dof18musc_inverse"
    assert _backend(configs.double_pendulum(4)) == "generated:double_pendulum"
    # kinematic constraints (CoordinateCoupler multipliers, errors, slacks)
    assert _backend(configs.double_pendulum_coupled(4)) == "generated:coupled_pendulum"
    assert _backend(configs.rajagopal80(4)) == "generated:rajagopal80"
    assert _backend(configs.rajagopal18_inverse(4)) == "generated:rajagopal18_inverse"
    # muscle wrapping over cylinders (PathWraps kept)
    assert _backend(configs.wrapped_pendulum(4)) == "generated:wrapped_pendulum"
    assert _backend(configs.rajagopal80(4, keep_path_wraps=True)) == "generated:rajagopal80_wrapped"
    assert _backend(configs.rajagopal18_inverse(4, keep_path_wraps=True)) == \
        "generated:rajagopal18_inverse_wrapped"
    # the wrap geometry is run-time data: another quadrant / radius / offset
    # keeps the code
    for quad in ("+x", "-y"):
        assert _backend(configs.wrapped_pendulum(4, quadrant=quad)) == "generated:wrapped_pendulum"
    st = configs.rajagopal80(4, keep_path_wraps=True)
    for w in st.problem.model.wraps.values():
        w.radius *= 1.05
        w.translation = tuple(x + 0.001 for x in w.translation)
    assert _backend(st) == "generated:rajagopal80_wrapped"
    # other constraint-derivative settings than generated: the interpreter
    assert _backend(configs.double_pendulum_coupled(4, enforce_constraint_derivatives=False)).startswith(
        "generic")


def test_heavier_femur_keeps_the_generated_back_end():
    st = configs.gait10dof18musc(4)
    st.problem.model.bodies["femur_r"].mass *= 1.01
    assert _backend(st) == "generated:gait10dof18musc_rigid"


def test_scaled_subject_keeps_the_generated_back_end():
    for mk, want in ((lambda: configs.gait10dof18musc(4), "generated:gait10dof18musc_rigid"),
                     (lambda: configs.gait10dof18musc_inverse(4), "generated:gait10dof18musc_inverse")):
        st = mk()
        configs.scale_subject(st.problem.model, 1.04, 1.07)
        assert _backend(st) == want


def test_scaled_rajagopal_keeps_the_generated_back_end():
    st = configs.rajagopal80(4)
    configs.scale_subject(st.problem.model, 0.97, 0.92)
    assert _backend(st) == "generated:rajagopal80"
    st = configs.rajagopal18_inverse(4)
    configs.scale_subject(st.problem.model, 1.02, 1.1)
    assert _backend(st) == "generated:rajagopal18_inverse"


def test_other_trial_data_keeps_the_generated_back_end():
    """A GRF table of another length (another trial) fits the same code:
    segment counts and breakpoints are run-time data."""
    st = configs.gait10dof18musc(4)
    m = st.problem.model
    t = m.tables["grf"]
    keep = slice(0, len(t.times) - 37)
    t.times = np.asarray(t.times)[keep]
    t.columns = {k: np.asarray(v)[keep] for k, v in t.columns.items()}
    assert _backend(st) == "generated:gait10dof18musc_rigid"


def test_structural_change_falls_back_to_the_interpreter():
    from mocohip.model import PathPoint
    st = configs.gait10dof18musc(4)
    mu = st.problem.model.muscles[0]
    mu.points.insert(1, PathPoint(mu.points[0].body, (0.01, 0.02, 0.03)))
    assert _backend(st).startswith("generic")
    # a parameter the code folded as a structural zero becomes nonzero
    st = configs.gait10dof18musc(4)
    b = st.problem.model.bodies["femur_r"]
    assert b.com[0] == 0.0
    b.com = (0.01, b.com[1], b.com[2])
    assert _backend(st).startswith("generic")
    # a nonzero parameter becoming zero keeps the code (it multiplies by it)
    st = configs.gait10dof18musc(4)
    b = st.problem.model.bodies["femur_r"]
    b.com = (0.0, 0.0, 0.0)
    assert _backend(st) == "generated:gait10dof18musc_rigid"
