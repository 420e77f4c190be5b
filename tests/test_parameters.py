"""MocoParameter (Moco/Moco/MocoParameter.h:91-170, MocoParameter.cpp): NLP
variables after the grid blocks that write model properties (body mass,
mass center, inertia; spring stiffness / rest length / viscosity; actuator
optimal force; muscle max isometric force), and the reference's
testMocoParameters.cpp problems (the oscillator's mass; one parameter on two
springs' stiffness).

CPU: the oracle's parameter columns against a numerical derivative of its
own g, the structure covering every dependent row, the reference's solves
(mass / stiffness within epsilon 0.003), the host-only layout query
(mh_get_nlp_info_for) against the oracle's sizes, and the input checks.
GPU: the device's parameter path against the oracle (g, the Jacobian, the
structure bit for bit -- also the tests/test_gpu_parity.py matrix), shards,
the device solve."""
import ctypes as C

import numpy as np
import pytest

from mocohip import abi, configs
from mocohip.ipm import IpmOptions, solve_ipm
from mocohip.solver import OracleNLP
from mocohip.trajectory import MocoTrajectory

STUDIES = {
    "oscillator_mass": lambda: configs.oscillator_mass(10),
    "oscillator_two_springs": lambda: configs.oscillator_two_springs(8),
    "oscillator_mass_trap_backward": lambda: _fd(_scheme(configs.oscillator_mass(8), "trapezoidal"), "backward"),
    "oscillator_two_springs_implicit_central": lambda: _fd(_implicit(configs.oscillator_two_springs(6)),
                                                           "central"),
    "gait_parameters": lambda: configs.gait10dof18musc_parameters(3),
}


def _scheme(st, s):
    st.solver.transcription_scheme = s
    return st


def _fd(st, s):
    st.solver.optim_finite_difference_scheme = s
    return st


def _implicit(st):
    st.solver.multibody_dynamics_mode = "implicit"
    return st


def _dense(nlp, x):
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    return J, ir, jc


@pytest.mark.parametrize("name", list(STUDIES))
def test_oracle_parameter_columns_are_the_derivative_of_g(name):
    """Each parameter column of the oracle's Jacobian (forward / backward /
    central differences of the callbacks on a copy of the model with the
    property moved, MocoParameter::applyParameterToModelProperties) equals a
    central difference of g along that parameter, and the block-dense
    structure holds every row g depends on through it."""
    st = STUDIES[name]()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options(), threads=8)
    try:
        assert nlp.NPAR == len(st.problem.parameters)
        x = nlp.initial_guess_from_bounds()
        r = np.random.default_rng(3)
        lo, hi = nlp.bounds()[:2]
        XP = nlp.n - nlp.NPAR
        for p in range(nlp.NPAR):   # parameters off the bounds midpoint
            x[XP + p] = lo[XP + p] + (hi[XP + p] - lo[XP + p]) * r.uniform(0.3, 0.7)
        J, ir, jc = _dense(nlp, x)
        # the callbacks' forward differences (step fd_step on a parameter of
        # size up to 5e3) cancel to eps |F| / fd_step, F the largest DAE
        # output at the iterate (the bounds-midpoint gait state drives the
        # accelerations to ~1e5), scaled into the defects by the interval
        # length: the reference's quotient has the same rounding
        G = nlp.G
        mesh = np.linspace(0.0, 1.0, G)
        P = np.concatenate([((x[1] - x[0]) * mesh + x[0])[:, None], nlp.point_inputs(x)], 1)
        F = float(np.abs(nlp.eval_dae(P)).max())
        fd_round = 64 * np.finfo(float).eps * (F + 1.0) * (abs(x[1] - x[0]) + 1.0) / st.solver.fd_step
        for p in range(nlp.NPAR):
            c = XP + p
            step = 1e-4 * max(1.0, abs(x[c]))
            e = np.zeros(nlp.n)
            e[c] = step
            d = (nlp.eval_g(x + e) - nlp.eval_g(x - e)) / (2 * step)
            scale = np.abs(d).max() + 1.0
            assert np.abs(J[:, c] - d).max() <= 1e-4 * scale + fd_round, (p, np.abs(J[:, c] - d).max(), scale, fd_round)
            rows = set(ir[jc == c].tolist())
            dep = set(np.nonzero(np.abs(d) > 1e-9 * scale)[0].tolist())
            assert dep <= rows, sorted(dep - rows)[:10]
            assert len(rows) > 0
    finally:
        nlp.close()


@pytest.mark.parametrize("name,true,start", [("oscillator_mass", configs.OSCILLATOR_MASS, None),
                                             ("oscillator_mass", configs.OSCILLATOR_MASS, 3.0),
                                             ("oscillator_two_springs", 0.5 * configs.OSCILLATOR_STIFFNESS, None),
                                             ("oscillator_two_springs", 0.5 * configs.OSCILLATOR_STIFFNESS, 70.0)])
def test_oracle_solve_recovers_the_parameter(name, true, start):
    """testMocoParameters.cpp:95-98,162-165: the solution's parameter equals
    the value that makes the oscillator's half period the final time, within
    epsilon 0.003 -- from the reference's starting point (the bounds
    midpoint) and from a parameter guess away from the answer."""
    st = getattr(configs, name)(25)
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options(), threads=8)
    try:
        x0 = st.solver.starting_point(nlp)
        if start is not None:
            x0[-1] = start
        r = solve_ipm(nlp, x0, IpmOptions.from_ipopt(st.solver.ipopt_options()))
        assert r.success, r.status
        sol = MocoTrajectory.from_iterate(nlp, r.x)
        par = st.problem.parameters[0].name
        assert sol.get_parameter(par) == pytest.approx(true, rel=0.003)
        # the iterate round-trips through the trajectory, parameter included
        assert np.array_equal(sol.to_iterate(nlp)[-nlp.NPAR:], r.x[-nlp.NPAR:])
    finally:
        nlp.close()


@pytest.mark.parametrize("name", list(STUDIES) + ["gait_inverse"])
def test_layout_query_matches_the_oracle(name):
    """mh_get_nlp_info_for (host only, no device, no context) sizes n, m and
    the block-dense nonzeros exactly as the oracle lays the NLP out."""
    st = STUDIES[name]() if name in STUDIES else configs.gait10dof18musc_inverse(3, sparsity="none")
    rep = st.problem.create_rep()
    opts = st.solver.options()
    info = abi.mh_nlp_info()
    lib = abi.load_mocohip()
    assert lib.mh_get_nlp_info_for(C.byref(rep.struct), C.byref(opts), C.byref(info)) == 0, \
        lib.mh_last_error().decode()
    nlp = OracleNLP(rep, opts, threads=2)
    try:
        assert (int(info.n), int(info.m), int(info.nnz_jac_g)) == (nlp.n, nlp.m, nlp.nnz)
        assert (int(info.num_states), int(info.num_controls)) == (nlp.NS, nlp.NC)
    finally:
        nlp.close()


def test_parameter_input_checks():
    """MocoParameter::initializeOnModel's checks: a component that exists
    and owns the property, an element for (only) vector properties; names
    unique; detected sparsity is refused with parameters (both sides)."""
    cases = []
    st = configs.oscillator_mass(4)
    st.problem.parameters[0].property_name = "inertia"
    cases.append((st, ValueError, "needs an element in \\[0, 6\\)"))
    st = configs.oscillator_mass(4)
    st.problem.parameters[0].property_element = 0
    cases.append((st, ValueError, "a property element was given"))
    st = configs.oscillator_two_springs(4)
    st.problem.parameters[0].property_name = "mass"
    cases.append((st, ValueError, "has no property 'mass'"))
    st = configs.oscillator_two_springs(4)
    st.problem.parameters[0].property_name = "frequency"
    cases.append((st, NotImplementedError, "not a parameterizable property"))
    st = configs.oscillator_mass(4)
    st.problem.add_parameter("oscillator_mass", "body", "mass", (0, 10))
    cases.append((st, ValueError, "duplicate name"))
    st = configs.oscillator_mass(4)
    st.problem.parameters[0].component_paths = ["/bodyset/nobody"]
    cases.append((st, ValueError, "no component '/bodyset/nobody'"))
    for st, exc, msg in cases:
        with pytest.raises(exc, match=msg):
            st.problem.create_rep()
    st = configs.oscillator_mass(4)
    st.solver.optim_sparsity_detection = "random"
    with pytest.raises(RuntimeError, match="sparsity detection"):
        OracleNLP(st.problem.create_rep(), st.solver.options())


def test_parameter_targets_lowered():
    """The lowered targets: one per component path, each naming the
    parameter, the property kind, the component's index and the element."""
    st = configs.gait10dof18musc_parameters(2)
    rep = st.problem.create_rep()
    p = rep.struct
    assert p.nparameters == 4 and p.nparameter_targets == 6
    t = [(p.parameter_targets[i].parameter, p.parameter_targets[i].kind, p.parameter_targets[i].element)
         for i in range(6)]
    assert t == [(0, abi.MH_PARAM_BODY_MASS, 0), (0, abi.MH_PARAM_BODY_MASS, 0),
                 (1, abi.MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE, 0), (1, abi.MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE, 0),
                 (2, abi.MH_PARAM_BODY_MASS_CENTER, 1), (3, abi.MH_PARAM_ACTUATOR_OPTIMAL_FORCE, 0)]
    assert rep.parameter_names == ["femur_mass", "soleus_fmax", "torso_com_y", "pelvis_tilt_reserve"]
    bl = [(p.parameter_bounds[i].lower, p.parameter_bounds[i].upper) for i in range(4)]
    assert bl == [(5.0, 12.0), (2000.0, 5000.0), (0.25, 0.45), (1.0, 50.0)]


# ---- on the device ---------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", list(STUDIES))
def test_device_parameter_jacobian_matches_the_oracle(name):
    """Structure, bounds and guess bit for bit; g and the parameter columns
    of the Jacobian against the oracle (the model copies of the device's
    parameter lanes -- k_apply_params -- against the oracle's param_ctx)."""
    from mocohip.solver import HipNLP
    st = STUDIES[name]()
    rep = st.problem.create_rep()
    gpu = HipNLP(rep, st.solver.options())
    ref = OracleNLP(rep, st.solver.options(), threads=8)
    try:
        assert (gpu.n, gpu.m, gpu.nnz) == (ref.n, ref.m, ref.nnz)
        ir, jc = gpu.jac_structure()
        ir0, jc0 = ref.jac_structure()
        assert np.array_equal(ir, ir0) and np.array_equal(jc, jc0)
        for a, b in zip(gpu.bounds(), ref.bounds()):
            assert np.array_equal(a, b)
        x = ref.initial_guess_from_bounds()
        XP = gpu.n - gpu.NPAR
        x[XP:] *= 0.9
        g, g0 = gpu.eval_g(x), ref.eval_g(x)
        assert np.abs(g - g0).max() <= 1e-10 * (np.abs(g0).max() + 1.0)
        J, J0 = gpu.eval_jac_g(x), ref.eval_jac_g(x)
        # FD quotients of g-level rounding differences: |dg| / h
        dg = np.abs(g - g0).max() + 64 * np.finfo(float).eps * (np.abs(g0).max() + 1.0)
        tol = 1e-8 * np.abs(J0) + 8 * dg * (1.0 + np.abs(x[1] - x[0])) / st.solver.fd_step
        bad = np.abs(J - J0) > tol
        assert not bad.any(), (int(bad.sum()), float(np.abs(J - J0).max()))
        # the same iterate twice: bit-identical (the model copies are rebuilt
        # from the pristine model every call)
        assert np.array_equal(gpu.eval_jac_g(x), J) and np.array_equal(gpu.eval_g(x), g)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["oscillator_two_springs", "gait_parameters"])
def test_device_objective_first_call(name):
    """The objective and its gradient as a fresh context's FIRST calls (the
    optimizer's scaling pass, before any constraint evaluation): the goals
    read the model copy the iterate's parameters were applied to -- created
    as the pristine model and rewritten by every objective call -- and agree
    with the oracle."""
    from mocohip.solver import HipNLP
    st = STUDIES[name]()
    rep = st.problem.create_rep()
    ref = OracleNLP(rep, st.solver.options(), threads=8)
    for trial in range(2):
        gpu = HipNLP(rep, st.solver.options())
        try:
            x = ref.initial_guess_from_bounds()
            x[gpu.n - gpu.NPAR:] *= 0.8 + 0.1 * trial
            if trial == 0:
                gf, f = gpu.eval_grad_f(x), gpu.eval_f(x)
            else:
                f, gf = gpu.eval_f(x), gpu.eval_grad_f(x)
            f0, gf0 = ref.eval_f(x), ref.eval_grad_f(x)
            assert f == pytest.approx(f0, rel=1e-12, abs=1e-12)
            tol = 1e-8 * np.abs(gf0) + 1e3 * np.finfo(float).eps * max(abs(f0), 1.0) / st.solver.fd_step
            assert np.all(np.abs(gf - gf0) <= tol)
        finally:
            gpu.close()
    ref.close()


@pytest.mark.gpu
def test_device_parameter_shards_reassemble_bit_exact():
    """Mesh-interval shards with parameters (every shard holds the parameter
    columns of its rows) concatenate to the unsharded g and Jacobian."""
    from mocohip.solver import HipNLP
    st = configs.gait10dof18musc_parameters(6)
    rep = st.problem.create_rep()
    full = HipNLP(rep, st.solver.options())
    x = full.random_iterate(np.random.default_rng(2).uniform(-1, 1, full.n))
    g, J = full.eval_g(x), full.eval_jac_g(x)
    gs, Js = [], []
    for a, b in [(0, 2), (2, 5), (5, 6)]:
        sh = HipNLP(rep, st.solver.options(a, b))
        gs.append(sh.eval_g(x))
        Js.append(sh.eval_jac_g(x))
        sh.close()
    full.close()
    assert np.array_equal(np.concatenate(gs), g)
    assert np.array_equal(np.concatenate(Js), J)


@pytest.mark.gpu
@pytest.mark.parametrize("name,true", [("oscillator_mass", configs.OSCILLATOR_MASS),
                                       ("oscillator_two_springs", 0.5 * configs.OSCILLATOR_STIFFNESS)])
def test_device_solve_recovers_the_parameter(name, true):
    """testMocoParameters.cpp on the HIP path: MocoStudy.solve returns the
    parameter within epsilon 0.003."""
    st = getattr(configs, name)(25)
    sol = st.solve()
    assert sol.metadata["success"] == "true", sol.metadata
    assert sol.get_parameter(st.problem.parameters[0].name) == pytest.approx(true, rel=0.003)


def test_oracle_dae_with_parameters_applied():
    """orc_eval_dae_params (the oracle side of the device's parameter lanes):
    at the model's own property value it is the pristine DAE bit for bit;
    the oscillator's acceleration -k q / m scales with 1 / mass."""
    st = configs.oscillator_mass(4)
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    try:
        x = nlp.initial_guess_from_bounds()
        rows = np.array([[0.1, 0.3, -0.2, 0.0], [0.2, -0.4, 0.5, 0.0]])[:, :1 + nlp.NI]
        x[-1] = 0.5 * configs.OSCILLATOR_MASS   # the model's body mass
        assert np.array_equal(nlp.eval_dae_params(rows, x), nlp.eval_dae(rows))
        x[-1] = configs.OSCILLATOR_MASS
        a = nlp.eval_dae_params(rows, x)[:, 0]
        assert a == pytest.approx(-configs.OSCILLATOR_STIFFNESS * rows[:, 1] / configs.OSCILLATOR_MASS, rel=1e-14)
        b = nlp.eval_dae_params(rows, x, 0, 1.0)[:, 0]
        assert b == pytest.approx(-configs.OSCILLATOR_STIFFNESS * rows[:, 1] / (configs.OSCILLATOR_MASS + 1.0),
                                  rel=1e-14)
    finally:
        nlp.close()
