"""The BASELINE.json configurations as MocoStudy builders.

  sliding_mass        configs[0]: exampleSlidingMass (Moco/Examples/C++/
                      exampleSlidingMass/exampleSlidingMass.cpp:35-90)
  double_pendulum     configs[1]: ModelFactory::createNLinkPendulum(2)
                      (Moco/Moco/Components/ModelFactory.cpp:33-89) with the
                      bounds of testImplicit.cpp:63-75
  gait10dof18musc     configs[2]: MocoTrack gait10dof18musc
                      (Moco/Tests/testMocoTrack.cpp:46-68) with the muscles
                      replaced by DeGrooteFregly2016Muscle
                      (ModOpReplaceMusclesWithDeGrooteFregly2016) instead of
                      removed, plus ModOpAddReserves(100) and the GRF
                      ExternalLoads; MocoTrack settings from MocoTrack.cpp:54-132.
"""
from __future__ import annotations

import json
import math
import os
from typing import Optional

import numpy as np

from .model import (Body, Coordinate, CoordinateActuator, DataTable,
                    ExternalForce, Joint, Marker, Model, SpringGeneralizedForce, model_from_dict)
from . import abi
from .osim import add_reserves
from .problem import (Constant, GCVSpline, ImplicitAuxiliaryDerivativesTerm,
                      MocoControlBoundConstraint, MocoControlGoal, MocoInitialActivationGoal,
                      MocoFinalTimeGoal, MocoMarkerFinalGoal, MocoProblem, MocoStateTrackingGoal,
                      PiecewiseLinearFunction)
from .solver import MocoHipSolver, MocoStudy

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def sliding_mass(num_mesh_intervals: int = 50, dynamics: str = "explicit") -> MocoStudy:
    m = Model("sliding_mass", gravity=(0, 0, 0))
    m.add_body(Body("body", 2.0, (0, 0, 0), (0, 0, 0, 0, 0, 0)))
    pos = Coordinate("position", (-math.inf, math.inf), "translational", path="/slider/position")
    m.add_joint(Joint.slider("slider", "ground", "body", pos))
    m.add_coordinate_actuator(CoordinateActuator("actuator", "position", 1.0, path="/actuator"))
    p = MocoProblem(m)
    p.set_time_bounds(0.0, (0.0, 5.0))
    p.set_state_info("/slider/position/value", (-5, 5), 0, 1)
    p.set_state_info("/slider/position/speed", (-50, 50), 0, 0)
    p.set_control_info("/actuator", (-50, 50))
    p.add_goal(MocoFinalTimeGoal())
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


# testMocoParameters.cpp:34-37: the oscillator's true mass and stiffness
OSCILLATOR_STIFFNESS = 100.0
OSCILLATOR_MASS = 5.0
OSCILLATOR_FINAL_TIME = math.pi * math.sqrt(OSCILLATOR_MASS / OSCILLATOR_STIFFNESS)


def _oscillator(body_mass: float, springs) -> Model:
    """createOscillatorModel / createOscillatorTwoSpringsModel
    (testMocoParameters.cpp:38-58,103-133): a body on a SliderJoint
    ("slider", coordinate "position"), no gravity, SpringGeneralizedForce(s)
    on the coordinate, rest length 0, no viscosity; a marker at the body's
    origin stands for the test's FinalPositionGoal (below)."""
    m = Model("oscillator", gravity=(0, 0, 0))
    m.add_body(Body("body", body_mass, (0, 0, 0), (0, 0, 0, 0, 0, 0)))
    pos = Coordinate("position", (-math.inf, math.inf), "translational", path="/slider/position")
    m.add_joint(Joint.slider("slider", "ground", "body", pos))
    for name, k in springs:
        m.add_spring(SpringGeneralizedForce(name, "position", stiffness=k, rest_length=0.0, viscosity=0.0))
    m.add_marker(Marker("body_origin", "body", (0.0, 0.0, 0.0)))
    return m


def _oscillator_study(m: Model, num_mesh_intervals: int) -> MocoStudy:
    """The test's problem (testMocoParameters.cpp:81-94,141-156): time in [0,
    pi sqrt(MASS / STIFFNESS)], position starting at -0.5 and ending in [0.25,
    0.75], speed 0 at both ends, and FinalPositionGoal -- (final position -
    0.5)^2 (:60-72), here MocoMarkerFinalGoal of the body origin against (0.5,
    0, 0): the same cost, since the origin is at (q, 0, 0)."""
    p = MocoProblem(m)
    p.set_time_bounds(0, OSCILLATOR_FINAL_TIME)
    p.set_state_info("/slider/position/value", (-5.0, 5.0), -0.5, (0.25, 0.75))
    p.set_state_info("/slider/position/speed", (-20, 20), 0, 0)
    p.add_goal(MocoMarkerFinalGoal(name="final_position", point_name="/markerset/body_origin",
                                   reference_location=(0.5, 0.0, 0.0)))
    return MocoStudy(p, MocoHipSolver(num_mesh_intervals=num_mesh_intervals))


def oscillator_mass(num_mesh_intervals: int = 25) -> MocoStudy:
    """testMocoParameters.cpp:78-99 ("Oscillator mass"): the body starts at
    half the true mass; MocoParameter "oscillator_mass" writes the body's
    mass, bounds [0, 10]; the solve must recover MASS within 0.3 %."""
    st = _oscillator_study(_oscillator(0.5 * OSCILLATOR_MASS, [("spring", OSCILLATOR_STIFFNESS)]),
                           num_mesh_intervals)
    st.problem.add_parameter("oscillator_mass", "body", "mass", (0, 10))
    return st


def oscillator_two_springs(num_mesh_intervals: int = 25) -> MocoStudy:
    """testMocoParameters.cpp:135-166 ("One parameter two springs"): two
    springs of a quarter of the stiffness each, ONE MocoParameter
    "spring_stiffness" writing both (bounds [0, 100]); the solve must find
    half the stiffness within 0.3 %."""
    st = _oscillator_study(_oscillator(OSCILLATOR_MASS, [("spring1", 0.25 * OSCILLATOR_STIFFNESS),
                                                         ("spring2", 0.25 * OSCILLATOR_STIFFNESS)]),
                           num_mesh_intervals)
    st.problem.add_parameter("spring_stiffness", ["spring1", "spring2"], "stiffness", (0, 100))
    return st


def gait10dof18musc_parameters(num_mesh_intervals: int = 6, **kw) -> MocoStudy:
    """gait10dof18musc with MocoParameters over every property kind a
    muscle-driven gait model offers (MocoParameter.h:91-170; test case, no
    reference counterpart on this model): one parameter on both femurs'
    mass, both soleus' max_isometric_force, the torso's mass-center y (a
    vector-property element), a reserve actuator's optimal_force."""
    st = gait10dof18musc(num_mesh_intervals, **kw)
    p = st.problem
    p.add_parameter("femur_mass", ["/bodyset/femur_r", "/bodyset/femur_l"], "mass", (5.0, 12.0))
    p.add_parameter("soleus_fmax", ["/forceset/soleus_r", "/forceset/soleus_l"], "max_isometric_force",
                    (2000.0, 5000.0))
    p.add_parameter("torso_com_y", "/bodyset/torso", "mass_center", (0.25, 0.45), property_element=1)
    p.add_parameter("pelvis_tilt_reserve", "/forceset/reserve_jointset_ground_pelvis_pelvis_tilt",
                    "optimal_force", (1.0, 50.0))
    return st


def sliding_mass_interface(num_mesh_intervals: int = 19, scheme: str = "trapezoidal",
                           dynamics: str = "explicit") -> MocoStudy:
    """testMocoInterface.cpp:41-83 ("Sliding mass", :1701-1742): a 10 kg
    mass on a slider, control in [-10, 10] N, from x = 0 to x = 1 at rest,
    minimum final time in [0, 10], trapezoidal, 19 mesh intervals; the
    reference's solution is bang-bang with final time 2.0."""
    m = Model("sliding_mass", gravity=(0, 0, 0))
    m.add_body(Body("body", 10.0, (0, 0, 0), (0, 0, 0, 0, 0, 0)))
    pos = Coordinate("position", (-math.inf, math.inf), "translational", path="/slider/position")
    m.add_joint(Joint.slider("slider", "ground", "body", pos))
    m.add_coordinate_actuator(CoordinateActuator("actuator", "position", 1.0, -10.0, 10.0,
                                                 path="/actuator"))
    p = MocoProblem(m)
    p.set_time_bounds(0.0, (0.0, 10.0))
    p.set_state_info("/slider/position/value", (0, 1), 0, 1)
    p.set_state_info("/slider/position/speed", (-100, 100), 0, 0)
    p.add_goal(MocoFinalTimeGoal())
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics, enforce_constraint_derivatives=False)
    return MocoStudy(p, s)


def n_link_pendulum(num_links: int, inertia=(1, 1, 1, 0, 0, 0)) -> Model:
    """ModelFactory::createNLinkPendulum (inertia=(0,)*6: point masses at
    the link tips, tropter's double pendulum, test_double_pendulum.cpp:45-74)."""
    m = Model({1: "pendulum", 2: "double_pendulum"}.get(num_links, f"{num_links}_link_pendulum"))
    prev = "ground"
    for i in range(num_links):
        m.add_body(Body(f"b{i}", 1.0, (0, 0, 0), tuple(inertia)))
        q = Coordinate(f"q{i}", (-math.pi / 2, math.pi / 2))
        m.add_joint(Joint.pin(f"j{i}", prev, f"b{i}", q, loc_in_child=(-1, 0, 0)))
        prev = f"b{i}"
    for i in range(num_links):
        m.add_coordinate_actuator(CoordinateActuator(f"tau{i}", f"q{i}", 1.0, path=f"/tau{i}"))
    for i in range(num_links):   # ModelFactory.cpp:74-75: at each body's origin
        m.add_marker(Marker(f"marker{i}", f"b{i}", (0.0, 0.0, 0.0)))
    return m


def double_pendulum(num_mesh_intervals: int = 100, scheme: str = "hermite-simpson",
                    dynamics: str = "explicit") -> MocoStudy:
    """testImplicit.cpp:63-75 solves this problem in both dynamics modes."""
    m = n_link_pendulum(2)
    p = MocoProblem(m)
    p.set_time_bounds(0.0, (0.0, 5.0))
    p.set_state_info("/jointset/j0/q0/value", (-10, 10), 0)
    p.set_state_info("/jointset/j0/q0/speed", (-50, 50), 0, 0)
    p.set_state_info("/jointset/j1/q1/value", (-10, 10), 0)
    p.set_state_info("/jointset/j1/q1/speed", (-50, 50), 0, 0)
    p.set_control_info("/tau0", (-100, 100))
    p.set_control_info("/tau1", (-100, 100))
    p.add_goal(MocoFinalTimeGoal(weight=0.001))
    p.add_goal(MocoControlGoal(weight=1e-3))
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


def double_pendulum_coupled(num_mesh_intervals: int = 20, scheme: str = "hermite-simpson",
                           dynamics: str = "explicit", enforce_constraint_derivatives: bool = True,
                           coupler: str = "linear", minimize_multipliers: bool = True) -> MocoStudy:
    """testConstraints.cpp:620-690 (testDoublePendulumCoordinateCoupler): a
    CoordinateCouplerConstraint q1 = -2 q0 + pi (LinearFunction(-2, pi)),
    control goal, HS N=20, both dynamics modes, with and without enforcing
    the constraint derivatives, minimizing the Lagrange multipliers with
    weight 10.  coupler="spline":
    the same constraint through a SimmSpline of the linear relation plus a
    quadratic term, so that f'' != 0 (acceleration errors and the
    velocity-correction Jacobian see the curvature)."""
    from .model import CoordinateCouplerConstraint, Function
    m = n_link_pendulum(2)
    if coupler == "linear":
        f = Function.linear("q0", -2.0, math.pi)
    else:
        xs = np.linspace(-6.0, 6.0, 13)
        f = Function.simm_spline("q0", xs, -2.0 * xs + math.pi + 0.1 * xs * xs)
    m.add_constraint(CoordinateCouplerConstraint("q0_q1_coupler", "q1", f))
    p = MocoProblem(m)
    p.set_time_bounds(0.0, 1.0)
    p.set_state_info("/jointset/j0/q0/value", (-5, 5), 0, math.pi / 2)
    p.set_state_info("/jointset/j0/q0/speed", (-10, 10), 0, 0)
    p.set_state_info("/jointset/j1/q1/value", (-10, 10))
    p.set_state_info("/jointset/j1/q1/speed", (-5, 5), 0, 0)
    p.set_control_info("/tau0", (-50, 50))
    p.set_control_info("/tau1", (-50, 50))
    p.add_goal(MocoControlGoal())
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics,
                      enforce_constraint_derivatives=enforce_constraint_derivatives,
                      minimize_lagrange_multipliers=minimize_multipliers, lagrange_multiplier_weight=10.0)
    return MocoStudy(p, s)


def double_pendulum_swingup(num_mesh_intervals: int = 29, scheme: str = "trapezoidal",
                            dynamics: str = "explicit", point_masses: bool = False) -> MocoStudy:
    """testImplicit.cpp:30-100 (solveDoublePendulumSwingup): final-time goal
    (weight 0.001) + MocoMarkerFinalGoal on /markerset/marker1 to (0, 2, 0)
    (weight 1000), trapezoidal, N=29, both dynamics modes.  point_masses:
    tropter's pendulum (no link inertia; test_double_pendulum.cpp:80-150)."""
    m = n_link_pendulum(2, inertia=(0, 0, 0, 0, 0, 0) if point_masses else (1, 1, 1, 0, 0, 0))
    p = MocoProblem(m)
    p.set_time_bounds(0.0, (0.0, 5.0))
    p.set_state_info("/jointset/j0/q0/value", (-10, 10), 0)
    p.set_state_info("/jointset/j0/q0/speed", (-50, 50), 0, 0)
    p.set_state_info("/jointset/j1/q1/value", (-10, 10), 0)
    p.set_state_info("/jointset/j1/q1/speed", (-50, 50), 0, 0)
    p.set_control_info("/tau0", (-100, 100))
    p.set_control_info("/tau1", (-100, 100))
    p.add_goal(MocoFinalTimeGoal(weight=0.001))
    p.add_goal(MocoMarkerFinalGoal("final", weight=1000.0, point_name="/markerset/marker1",
                                   reference_location=(0.0, 2.0, 0.0)))
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


def pendulum_control_bound(num_mesh_intervals: int = 20, section: str = "lower",
                           scheme: str = "hermite-simpson",
                           dynamics: str = "explicit") -> MocoStudy:
    """The MocoControlBoundConstraint problems of testConstraints.cpp:1460-1540
    (ModelFactory::createPendulum): "lower" (Constant 0.1318 lower bound),
    "upper" (Constant 11.236 upper bound, free final time), "equality"
    (PiecewiseLinearFunction lower bound with equality_with_lower), and
    "both" (GCVSpline lower and Constant upper bound, two equations)."""
    m = n_link_pendulum(1)
    p = MocoProblem(m)
    c = p.add_path_constraint(MocoControlBoundConstraint())
    c.add_control_path("/tau0")
    if section == "upper":
        p.set_time_bounds(0.0, (0.1, 10.0))
        p.set_state_info("/jointset/j0/q0/value", (0, 1), 0, 0.53)
        p.set_state_info("/jointset/j0/q0/speed", (-10, 10), 0, 0)
        p.set_control_info("/tau0", (-20, 20))
        p.add_goal(MocoFinalTimeGoal())
        c.set_upper_bound(Constant(11.236))
    else:
        p.set_time_bounds(0.0, 1.0)
        p.set_state_info("/jointset/j0/q0/value", (-10, 10), 0)
        p.set_state_info("/jointset/j0/q0/speed", (-10, 10), 0)
        p.set_control_info("/tau0", (-5, 5))
        p.add_goal(MocoControlGoal())
        if section == "lower":
            c.set_lower_bound(Constant(0.1318))
        elif section == "equality":
            c.set_lower_bound(PiecewiseLinearFunction([0, 0.2, 0.7, 1], [0, 0.5316, -0.3137, 0.0319]))
            c.set_equality_with_lower(True)
        elif section == "both":
            c.set_lower_bound(GCVSpline(5, [0, 0.2, 0.45, 0.7, 0.85, 1.0],
                                        [-0.4, 0.1, -0.2, 0.3, 0.0, -0.1]))
            c.set_upper_bound(Constant(2.5))
        else:
            raise ValueError(section)
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


def _load(name):
    with open(os.path.join(DATA, name)) as fh:
        return json.load(fh)


def gait10dof18musc_model(muscles: bool = True, tendon_compliance: bool = False,
                          reserves: float = 100.0, external_loads: bool = True,
                          tendon_dynamics: str = "explicit") -> Model:
    """tendon_dynamics: DeGrooteFregly2016Muscle tendon_compliance_dynamics_mode
    of the compliant tendons ("implicit": the MocoInverse test setting,
    ModOpTendonComplianceDynamicsModeDGF("implicit"), testMocoInverse.cpp:127)."""
    m = model_from_dict(_load("gait10dof18musc.json"))
    if not muscles:
        m.actuators = [a for a in m.actuators if not hasattr(a, "points")]
        m.muscles = []
    for mu in m.muscles:
        mu.ignore_tendon_compliance = not tendon_compliance
        mu.tendon_compliance_dynamics_mode = tendon_dynamics
    if reserves:
        add_reserves(m, reserves)
    if external_loads:
        grf = _load("walk_gait1018_subject01_grf.json")
        cols = {k: np.asarray(v) for k, v in grf["columns"].items()}
        m.add_table(DataTable("grf", np.asarray(grf["time"]), cols, degree=3))
        for ef in grf["external_forces"]:
            if ef["force_expressed_in_body"] != "ground" or ef["point_expressed_in_body"] != "ground":
                raise NotImplementedError("ExternalForce must be expressed in ground")
            m.add_external_force(ExternalForce(ef["name"], ef["body"], "grf",
                                               ef["force_identifier"], ef["point_identifier"],
                                               ef["torque_identifier"]))
    return m


def gait10dof18musc(num_mesh_intervals: int = 200, muscles: bool = True,
                    tendon_compliance: bool = False,
                    fd_scheme: str = "forward", dynamics: str = "explicit",
                    control_bounds: bool = False, tendon_dynamics: str = "explicit") -> MocoStudy:
    """MocoTrack gait10dof18musc (config 3).  MocoTrack: states tracking goal
    (weight 1, GCVSpline reference), control effort goal (0.001), time
    [0.01, 1.3], explicit dynamics, forward FD (MocoTrack.cpp:54-132).
    control_bounds: adds a MocoControlBoundConstraint on the soleus and
    tibialis anterior excitations (GCVSpline lower, Constant upper bound) and
    one on the hip flexor reserve (Constant upper bound) as path constraints
    (not part of the reference MocoTrack setup)."""
    m = gait10dof18musc_model(muscles=muscles, tendon_compliance=tendon_compliance,
                              tendon_dynamics=tendon_dynamics)
    ref = _load("walk_gait1018_state_reference.json")
    cols = {k: np.asarray(v) for k, v in ref["columns"].items()}
    m.add_table(DataTable("state_reference", np.asarray(ref["time"]), cols, degree=5))
    p = MocoProblem(m)
    p.add_goal(MocoStateTrackingGoal("state_tracking", 1.0, DataTable(
        "state_reference", np.asarray(ref["time"]), cols, degree=5)))
    p.add_goal(MocoControlGoal("control_effort", 0.001))
    p.set_time_bounds(0.01, 1.3)
    if control_bounds:
        names = m.control_names()
        picks = [n for n in names if n.endswith(("soleus_r", "tib_ant_r"))] if muscles else []
        c = p.add_path_constraint(MocoControlBoundConstraint("excitation_band"))
        for n in picks:
            c.add_control_path(n)
        c.set_lower_bound(GCVSpline(5, np.linspace(0.0, 1.4, 8),
                                    0.02 + 0.01 * np.sin(np.linspace(0.0, 3.0, 8))))
        c.set_upper_bound(Constant(0.9))
        r = p.add_path_constraint(MocoControlBoundConstraint("reserve_cap"))
        r.add_control_path(names[-1])
        r.set_upper_bound(Constant(0.5))
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals,
                      optim_finite_difference_scheme=fd_scheme, multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


def scale_subject(m: Model, length: float = 1.03, mass: float = 1.05) -> Model:
    """A scaled subject (what OpenSim's ScaleTool produces from a generic
    model, uniformly): every length -- joint frame locations, centers of
    mass, path-point locations, CustomJoint translation splines and
    MovingPathPoint functions, optimal fiber and tendon slack lengths --
    times ``length``,
    masses times ``mass``, inertias times mass * length^2.  The model
    STRUCTURE is unchanged, so a generated back end of the generic model
    serves it (codegen.py "Structure-only specialization")."""
    L, W = float(length), float(mass)
    for b in m.bodies.values():
        b.mass *= W
        b.com = tuple(L * c for c in b.com)
        b.inertia = tuple(W * L * L * i for i in b.inertia)
    for j in m.joints:
        j.loc_in_parent = tuple(L * c for c in j.loc_in_parent)
        j.loc_in_child = tuple(L * c for c in j.loc_in_child)
        for ax in j.axes:
            # translations that are functions of a rotation (the knee's
            # SimmSplines, MultiplierFunction); a translational coordinate's
            # own linear function is a length already
            if (ax.type == abi.MH_AXIS_TRANSLATION and ax.func is not None
                    and ax.func.kind != abi.MH_FN_LINEAR):
                ax.func = ax.func.scaled(L)
    for mu in m.muscles:
        mu.optimal_fiber_length *= L
        mu.tendon_slack_length *= L
        for pt in mu.points:
            pt.loc = tuple(L * c for c in pt.loc)
            pt.fx, pt.fy, pt.fz = (f.scaled(L) if f is not None else None for f in (pt.fx, pt.fy, pt.fz))
    return m


def gait10dof18musc_track(num_mesh_intervals: int = 65, muscles: bool = False) -> MocoStudy:
    """The reference's MocoTrack golden-solution problem (testMocoTrack.cpp:
    46-68): gait10dof18musc | ModOpRemoveMuscles | ModOpAddReserves(100) |
    ModOpAddExternalLoads; states reference walk_gait1018_state_reference.mot
    | TabOpLowPassFilter(6) tracked with weight 1 (GCVSpline of degree 5),
    control effort 0.001, time [0.01, 1.3], mesh_interval 0.02 (N = 65),
    explicit dynamics, forward differences, convergence and constraint
    tolerances 1e-2, bounds guess (MocoTrack.cpp:54-132).  Its converged
    solution is std_testMocoTrackGait10dof18musc_solution.sto.

    muscles=True: BASELINE configs[2], the same MocoTrack with the 18
    muscles replaced by DeGrooteFregly2016Muscle (rigid tendons,
    ModOpReplaceMusclesWithDeGrooteFregly2016) instead of removed -- the
    muscle-driven workload the headline throughput is measured on, solved
    with MocoTrack's settings."""
    from .splines import filter_lowpass_table
    m = gait10dof18musc_model(muscles=muscles)
    ref = _load("walk_gait1018_state_reference.json")
    tp, cols = filter_lowpass_table(ref["time"], {k: np.asarray(v) for k, v in ref["columns"].items()}, 6.0)
    m.add_table(DataTable("state_reference", tp, cols, degree=5))
    p = MocoProblem(m)
    p.add_goal(MocoStateTrackingGoal("state_tracking", 1.0, DataTable("state_reference", tp, cols, degree=5)))
    p.add_goal(MocoControlGoal("control_effort", 0.001))
    p.set_time_bounds(0.01, 1.3)
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, optim_finite_difference_scheme="forward",
                      optim_convergence_tolerance=1e-2, optim_constraint_tolerance=1e-2)
    return MocoStudy(p, s)


def gait10dof18musc_inverse(num_mesh_intervals: int = 25, fd_scheme: str = "forward",
                            sparsity: str = "random", subject=None) -> MocoStudy:
    """MocoInverse on gait10dof18musc (configs[4], one solve of the batch):
    kinematics prescribed by a PositionMotion of the coordinate trajectories
    (MocoInverse.cpp:46-66; GCVSpline degree 5, PositionMotion.cpp:121-155),
    DeGrooteFregly2016 muscles with compliant tendons in implicit mode
    (testMocoInverse.cpp:120-130), reserves, ExternalLoads, control effort
    goal with reserves weight 1 (MocoInverse.cpp:89-90), the initial-
    activation endpoint constraint (MocoInverse.cpp:93), implicit dynamics,
    no control-midpoint interpolation, forward differences and "random"
    sparsity detection (MocoInverse.cpp:104-114).  The kinematics are the
    bundled walking coordinate trajectories, clipped by 1e-3 at both ends
    (clip_time_range, MocoInverse.cpp:82-86).  ``subject`` = (length,
    mass) scales the model (scale_subject: one subject of a configs[4]
    sweep; the same kinematics)."""
    m = gait10dof18musc_model(tendon_compliance=True, tendon_dynamics="implicit")
    if subject is not None:
        m = scale_subject(m, *subject)
    ref = _load("walk_gait1018_state_reference.json")
    t = np.asarray(ref["time"])
    kin = DataTable("kinematics", t, {k: np.asarray(v) for k, v in ref["columns"].items()
                                      if k.endswith("/value")}, degree=5)
    p = MocoProblem(m)
    p.set_position_motion(kin)
    p.set_time_bounds(float(t[0]) + 1e-3, float(t[-1]) - 1e-3)
    p.add_goal(MocoControlGoal("excitation_effort", 1.0))
    # prevent "free" activation at the beginning of the motion (MocoInverse.cpp:93)
    p.add_goal(MocoInitialActivationGoal("initial_activation"))
    # minimize_implicit_auxiliary_derivatives, weight 0.01 (MocoInverse.cpp:106-107)
    p.add_goal(ImplicitAuxiliaryDerivativesTerm(weight=0.01))
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals,
                      optim_finite_difference_scheme=fd_scheme, multibody_dynamics_mode="implicit",
                      interpolate_control_midpoints=False,   # MocoInverse.cpp:105
                      optim_sparsity_detection=sparsity,
                      # MocoInverse convergence / constraint tolerance
                      # defaults (MocoInverse.cpp:38-39, 108-109)
                      optim_convergence_tolerance=1e-3, optim_constraint_tolerance=1e-3)
    return MocoStudy(p, s)


def wrapped_pendulum(num_mesh_intervals: int = 20, scheme: str = "hermite-simpson",
                     dynamics: str = "explicit", tendon_compliance: bool = False,
                     quadrant: str = "all") -> MocoStudy:
    # (compliant tendon: the angle range over which the path wraps, with
    # tendon slack and fiber lengths that keep the muscle near its optimal
    # fiber length there, so the explicit tendon dynamics stay regular)
    """A one-link pendulum (ModelFactory::createNLinkPendulum(1)) driven by a
    DeGrooteFregly2016 muscle whose path wraps over a WrapCylinder about the
    pin axis (the GeometryPath / WrapCylinder geometry of SURVEY §8 A9 on a
    model small enough for every kernel variant).  Not a BASELINE config."""
    from .model import DeGrooteFregly2016Muscle, PathPoint, WrapCylinder
    m = n_link_pendulum(1)
    m.add_wrap(WrapCylinder("pin_cyl", "ground", 0.1, 0.2, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), quadrant))
    mu = DeGrooteFregly2016Muscle("flexor", [PathPoint("ground", (-0.3, 0.15, 0.05), name="origin"),
                                             PathPoint("b0", (-0.7, 0.12, -0.04), name="insertion")],
                                  max_isometric_force=200.0,
                                  optimal_fiber_length=0.22 if tendon_compliance else 0.2,
                                  tendon_slack_length=0.45 if tendon_compliance else 0.25,
                                  pennation_angle_at_optimal=0.1,
                                  path_wraps=[("pin_cyl", -1, -1)])
    mu.ignore_tendon_compliance = not tendon_compliance
    m.actuators = [a for a in m.actuators]
    m.add_muscle(mu)
    p = MocoProblem(m)
    p.set_time_bounds(0.0, 1.0)
    p.set_state_info("/jointset/j0/q0/value", (-1.0, -0.4) if tendon_compliance else (-1.5, 1.5),
                     -0.7 if tendon_compliance else 0.5)
    p.set_state_info("/jointset/j0/q0/speed", (-3, 3), 0)
    p.set_control_info("/tau0", (-50, 50))
    p.add_goal(MocoControlGoal())
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      multibody_dynamics_mode=dynamics)
    return MocoStudy(p, s)


def _walk_armless_grf(m: Model):
    """ModOpAddExternalLoads(subject_walk_armless_external_loads.xml / grf_walk.xml):
    ground-expressed force, point and torque on calcn_r / calcn_l."""
    grf = _load("subject_walk_armless_grf.json")
    cols = {k: np.asarray(v) for k, v in grf["columns"].items()}
    m.add_table(DataTable("grf", np.asarray(grf["time"]), cols, degree=3))
    for ef in grf["external_forces"]:
        if ef["force_expressed_in_body"] != "ground" or ef["point_expressed_in_body"] != "ground":
            raise NotImplementedError("ExternalForce must be expressed in ground")
        m.add_external_force(ExternalForce(ef["name"], ef["body"], "grf", ef["force_identifier"],
                                           ef["point_identifier"], ef["torque_identifier"]))


def _walk_armless_kinematics(m: Model, lowpass: float = 6.0) -> DataTable:
    """TableProcessor("subject_walk_armless_coordinates.mot") |
    TabOpLowPassFilter(6), in radians, columns renamed to the model's
    coordinate value paths (extra columns dropped: kinematics_allow_extra_columns)."""
    from .splines import filter_lowpass_table
    kin = _load("subject_walk_armless_coordinates.json")
    byname = {c.name: c for c in m.coordinates()}
    cols = {byname[k].path + "/value": np.asarray(v) for k, v in kin["columns"].items() if k in byname}
    tp, fcols = filter_lowpass_table(kin["time"], cols, lowpass)
    return DataTable("kinematics", tp, fcols, degree=5)


def _replaced(m: Model, keep_path_wraps: bool = False) -> Model:
    """ModOpReplaceMusclesWithDeGrooteFregly2016 on a model stored with its
    Millard muscles' PathWrapSets: replaceMuscles copies the path points only
    (DeGrooteFregly2016Muscle.cpp:1007-1020), so the wraps go."""
    if not keep_path_wraps:
        for mu in m.muscles:
            mu.path_wraps = []
    return m


def rajagopal18_model(keep_path_wraps: bool = False) -> Model:
    """testMocoInverse.cpp:121-128: subject_walk_armless_18musc.osim |
    ModOpReplaceJointsWithWelds(subtalar, mtp) | ModOpReplaceMusclesWith
    DeGrooteFregly2016 | ModOpIgnorePassiveFiberForcesDGF |
    ModOpTendonComplianceDynamicsModeDGF("implicit") | ModOpAddExternalLoads.
    18 muscles over 16 PathWraps on WrapCylinders, 2 patellofemoral
    CoordinateCouplerConstraints, the model's own reserve actuators."""
    m = _replaced(model_from_dict(_load("rajagopal18.json")), keep_path_wraps)
    m.replace_joints_with_welds(["subtalar_r", "subtalar_l", "mtp_r", "mtp_l"])
    for mu in m.muscles:
        mu.ignore_passive_fiber_force = True
        mu.tendon_compliance_dynamics_mode = "implicit"
    _walk_armless_grf(m)
    return m


def rajagopal18_inverse(num_mesh_intervals: int = 11, fd_scheme: str = "forward",
                        sparsity: str = "random", keep_path_wraps: bool = False) -> MocoStudy:
    """MocoInverse Rajagopal2016, 18 muscles (testMocoInverse.cpp:118-147):
    time [0.45, 1.0], mesh_interval 0.05 (N = 11), kinematics low-pass
    filtered at 6 Hz and prescribed by a PositionMotion, the MocoInverse
    goals and solver settings (MocoInverse.cpp:46-120; see
    gait10dof18musc_inverse).  The coupler multipliers stay NLP variables
    (constraint forces in the residual), without kinematic rows.  Its
    converged solution is std_testMocoInverse_subject_18musc_solution.sto.
    keep_path_wraps=True keeps the Millard muscles' PathWraps (16 on
    WrapCylinders), which the reference's replaceMuscles drops."""
    m = rajagopal18_model(keep_path_wraps)
    kin = _walk_armless_kinematics(m)
    p = MocoProblem(m)
    p.set_position_motion(kin)
    p.set_time_bounds(0.45, 1.0)
    p.add_goal(MocoControlGoal("excitation_effort", 1.0))
    p.add_goal(MocoInitialActivationGoal("initial_activation"))
    p.add_goal(ImplicitAuxiliaryDerivativesTerm(weight=0.01))
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals,
                      optim_finite_difference_scheme=fd_scheme, multibody_dynamics_mode="implicit",
                      interpolate_control_midpoints=False, optim_sparsity_detection=sparsity,
                      optim_convergence_tolerance=1e-3, optim_constraint_tolerance=1e-3)
    return MocoStudy(p, s)


def rajagopal80_model(keep_path_wraps: bool = False) -> Model:
    """example3DWalking muscleDrivenStateTracking (exampleMocoTrack.cpp):
    subject_walk_armless.osim | ModOpAddExternalLoads(grf_walk.xml) |
    ModOpIgnoreTendonCompliance | ModOpReplaceMusclesWithDeGrooteFregly2016 |
    ModOpIgnorePassiveFiberForcesDGF | ModOpScaleActiveFiberForceCurveWidthDGF(1.5):
    80 DGF muscles (rigid tendons; their 46 PathWraps dropped by
    replaceMuscles unless keep_path_wraps), 18 coordinates, 2 patellofemoral
    couplers, the model's 6 pelvis actuators."""
    m = _replaced(model_from_dict(_load("rajagopal80.json")), keep_path_wraps)
    for mu in m.muscles:
        mu.ignore_tendon_compliance = True
        mu.ignore_passive_fiber_force = True
        mu.active_force_width_scale = 1.5
    _walk_armless_grf(m)
    return m


def rajagopal80(num_mesh_intervals: int = 400, fd_scheme: str = "forward",
                scheme: str = "hermite-simpson", keep_path_wraps: bool = False) -> MocoStudy:
    """BASELINE configs[3]: the Rajagopal 80-muscle gait NLP at N = 400.  The
    reference's 80-muscle problem (example3DWalking exampleMocoTrack.cpp
    muscleDrivenStateTracking: states tracking weight 10, control effort,
    time [0.81, 1.65], explicit dynamics with the patellofemoral couplers
    and their derivatives enforced, forward FD) on the filtered coordinate
    trajectories; BASELINE names a predictive problem, whose contact models
    are outside this path, so the goals here are the tracking example's
    (the NLP's layout, DAE and Jacobian are the same).  Block-dense callback
    sparsity (detection with kinematic constraints is rejected: SURVEY §8
    F2 note in DESIGN.md).  keep_path_wraps=True: with the 46 PathWraps."""
    m = rajagopal80_model(keep_path_wraps)
    kin = _walk_armless_kinematics(m)
    m.add_table(DataTable("state_reference", kin.times, kin.columns, degree=5))
    p = MocoProblem(m)
    p.add_goal(MocoStateTrackingGoal("state_tracking", 10.0, DataTable(
        "state_reference", kin.times, kin.columns, degree=5)))
    p.add_goal(MocoControlGoal("control_effort", 1.0))
    p.set_time_bounds(0.81, 1.65)
    s = MocoHipSolver(num_mesh_intervals=num_mesh_intervals, transcription_scheme=scheme,
                      optim_finite_difference_scheme=fd_scheme)
    return MocoStudy(p, s)


CONFIGS = {
    "sliding_mass": sliding_mass,
    "double_pendulum": double_pendulum,
    "double_pendulum_swingup": double_pendulum_swingup,
    "double_pendulum_coupled": double_pendulum_coupled,
    "gait10dof18musc": gait10dof18musc,
    "gait10dof18musc_inverse": gait10dof18musc_inverse,
    "gait10dof18musc_track": gait10dof18musc_track,
    "wrapped_pendulum": wrapped_pendulum,
    "rajagopal18_inverse": rajagopal18_inverse,
    "rajagopal80": rajagopal80,
}
