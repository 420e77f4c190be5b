"""MocoProblem / MocoProblemRep mirror: goals, bounds rules, and lowering of
a problem to the C-ABI ``mh_problem`` struct.

Default-bound rules restate MocoProblemRep::initialize
(Moco/Moco/MocoProblemRep.cpp:306-427) and MocoPhase defaults
(Moco/Moco/MocoProblem.cpp:30-43).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .model import CompiledModel, CoordinateActuator, DataTable, \
    DeGrooteFregly2016Muscle, Model, SpringGeneralizedForce
from .splines import gcv_interpolating_ppoly

NAN = float("nan")


@dataclass
class MocoBounds:
    lower: float = NAN
    upper: float = NAN

    @staticmethod
    def of(b) -> "MocoBounds":
        if b is None:
            return MocoBounds()
        if isinstance(b, MocoBounds):
            return b
        if isinstance(b, (int, float)):
            return MocoBounds(float(b), float(b))
        lo, hi = b
        return MocoBounds(float(lo), float(hi))

    def is_set(self) -> bool:
        return not (math.isnan(self.lower) or math.isnan(self.upper))


@dataclass
class MocoVariableInfo:
    bounds: MocoBounds = field(default_factory=MocoBounds)
    initial: MocoBounds = field(default_factory=MocoBounds)
    final: MocoBounds = field(default_factory=MocoBounds)


# ---------------------------------------------------------------- goals ----
@dataclass
class MocoControlGoal:
    """MocoControlGoal (Moco/Moco/MocoGoal/MocoControlGoal.cpp:54-131)."""
    name: str = "control_effort"
    weight: float = 1.0
    exponent: int = 2
    control_weights: Dict[str, float] = field(default_factory=dict)


@dataclass
class MocoStateTrackingGoal:
    """MocoStateTrackingGoal (MocoStateTrackingGoal.cpp:27-117).  The
    reference is a DataTable whose column labels are state paths."""
    name: str = "state_tracking"
    weight: float = 1.0
    reference: Optional[DataTable] = None
    state_weights: Dict[str, float] = field(default_factory=dict)


@dataclass
class MocoFinalTimeGoal:
    name: str = "final_time"
    weight: float = 1.0


@dataclass
class MocoSumSquaredStateGoal:
    name: str = "sum_squared_state"
    weight: float = 1.0
    state_weights: Dict[str, float] = field(default_factory=dict)


@dataclass
class MocoInitialActivationGoal:
    """MocoInitialActivationGoal (Moco/Moco/MocoGoal/MocoInitialActivationGoal.
    {h,cpp}): for every muscle with activation dynamics, the initial
    excitation equals the initial activation.  An endpoint constraint by
    default (getDefaultModeImpl, .h:40-42; MocoGoal.h:254-271 sets the weight
    to 1 in that mode); one equation per muscle in model order
    (initializeOnModelImpl, .cpp:23-39), bounds [0, 0]
    (MocoConstraintInfo.h:44-54)."""
    name: str = "initial_activation"
    mode: str = "endpoint_constraint"
    weight: float = 1.0


@dataclass
class MocoMarkerFinalGoal:
    """MocoMarkerFinalGoal (Moco/Moco/MocoGoal/MocoMarkerFinalGoal.{h,cpp}):
    cost = |location in ground of ``point_name`` at the final state -
    ``reference_location``|^2 (calcGoalImpl, .cpp:29-34; realizes Position
    only, so it depends on the final coordinates), times the weight."""
    name: str = "marker_final"
    weight: float = 1.0
    point_name: str = ""
    reference_location: Sequence[float] = (0.0, 0.0, 0.0)


# ------------------------------------------------- functions of time ----
@dataclass
class Constant:
    """OpenSim::Constant."""
    value: float

    def ppoly(self):
        return None


@dataclass
class PiecewiseLinearFunction:
    """OpenSim::PiecewiseLinearFunction: linear between points, extended
    linearly with the end segments' slopes."""
    x: Sequence[float]
    y: Sequence[float]

    def ppoly(self):
        x, y = np.asarray(self.x, float), np.asarray(self.y, float)
        if len(x) < 2 or np.any(np.diff(x) <= 0):
            raise ValueError("PiecewiseLinearFunction needs >= 2 increasing points")
        coefs = np.zeros((len(x) - 1, 1, 2))
        coefs[:, 0, 0] = y[:-1]
        coefs[:, 0, 1] = np.diff(y) / np.diff(x)
        return x, coefs


@dataclass
class GCVSpline:
    """OpenSim::GCVSpline through (x, y) (interpolating; splines.py)."""
    degree: int
    x: Sequence[float]
    y: Sequence[float]

    def ppoly(self):
        return gcv_interpolating_ppoly(np.asarray(self.x, float), np.asarray(self.y, float),
                                       int(self.degree))


# ----------------------------------------------------- path constraints ----
@dataclass
class MocoControlBoundConstraint:
    """MocoControlBoundConstraint (Moco/Moco/MocoControlBoundConstraint.cpp):
    lower_bound(t) <= control <= upper_bound(t) for each control path, as
    path-constraint equations control - bound(t) at every mesh point."""
    name: str = "control_bound"
    control_paths: List[str] = field(default_factory=list)
    lower_bound: Optional[object] = None
    upper_bound: Optional[object] = None
    equality_with_lower: bool = False

    def add_control_path(self, path: str):
        self.control_paths.append(path)

    def set_lower_bound(self, f):
        self.lower_bound = f

    def set_upper_bound(self, f):
        self.upper_bound = f

    def set_equality_with_lower(self, v: bool):
        self.equality_with_lower = bool(v)


@dataclass
class ImplicitAuxiliaryDerivativesTerm:
    """MocoDirectCollocationSolver minimize_implicit_auxiliary_derivatives /
    implicit_auxiliary_derivatives_weight as an objective term
    (CasOCTranscription.cpp:534-545): weight * integral of the sum of squared
    implicit auxiliary derivatives."""
    name: str = "auxiliary_derivatives"
    weight: float = 1.0


@dataclass
class MocoParameter:
    """MocoParameter (Moco/Moco/MocoParameter.h:91-170): an NLP variable
    written into the property ``property_name`` of every component in
    ``component_paths`` before each evaluation; ``property_element`` picks
    the element of a vector property (mass_center: 0-2, inertia: 0-5 = xx yy
    zz xy xz yz), -1 for a scalar one.  Components are named by name or path
    (a Body, SpringGeneralizedForce, CoordinateActuator or DGF muscle);
    supported properties: Body mass / mass_center / inertia,
    SpringGeneralizedForce stiffness / rest_length / viscosity,
    CoordinateActuator optimal_force, muscle max_isometric_force
    (include/mocohip.h mh_parameter_kind)."""
    name: str
    component_paths: Sequence[str]
    property_name: str
    bounds: MocoBounds = field(default_factory=MocoBounds)
    property_element: int = -1


class MocoProblem:
    """Single-phase MocoProblem (MocoProblem.h)."""

    def __init__(self, model: Optional[Model] = None):
        self.model = model
        self.time_initial = MocoBounds()
        self.time_final = MocoBounds()
        self.state_infos: Dict[str, MocoVariableInfo] = {}
        self.control_infos: Dict[str, MocoVariableInfo] = {}
        self.goals: List[object] = []
        self.path_constraints: List[object] = []
        self.position_motion: Optional[DataTable] = None
        self.default_speed_bounds = MocoBounds(-50.0, 50.0)
        self.bound_activation_from_excitation = True
        # MocoPhase kinematic_constraint_bounds / multiplier_bounds
        # (MocoProblem.cpp:42-43)
        self.kinematic_constraint_bounds = MocoBounds(0.0, 0.0)
        self.multiplier_bounds = MocoBounds(-1000.0, 1000.0)
        self.parameters: List[MocoParameter] = []

    def set_model(self, model: Model):
        self.model = model

    def set_kinematic_constraint_bounds(self, bounds):
        self.kinematic_constraint_bounds = MocoBounds.of(bounds)

    def set_multiplier_bounds(self, bounds):
        self.multiplier_bounds = MocoBounds.of(bounds)

    def set_time_bounds(self, initial, final):
        self.time_initial = MocoBounds.of(initial)
        self.time_final = MocoBounds.of(final)

    def set_state_info(self, name, bounds=None, initial=None, final=None):
        self.state_infos[name] = MocoVariableInfo(
            MocoBounds.of(bounds), MocoBounds.of(initial), MocoBounds.of(final))

    def set_control_info(self, name, bounds=None, initial=None, final=None):
        self.control_infos[name] = MocoVariableInfo(
            MocoBounds.of(bounds), MocoBounds.of(initial), MocoBounds.of(final))

    def add_parameter(self, name: str, component_paths, property_name: str, bounds=None,
                      property_element: int = -1) -> MocoParameter:
        """MocoProblem::addParameter (MocoProblem.h: the MocoParameter
        constructors, MocoParameter.h:100-112)."""
        paths = [component_paths] if isinstance(component_paths, str) else list(component_paths)
        par = MocoParameter(name, paths, property_name, MocoBounds.of(bounds), int(property_element))
        self.parameters.append(par)
        return par

    def add_goal(self, goal):
        self.goals.append(goal)
        return goal

    def set_position_motion(self, kinematics: DataTable):
        """PositionMotion::createFromTable (Components/PositionMotion.cpp:
        121-155): every coordinate prescribed by a GCVSpline (degree 5 unless
        the table says otherwise) of the column named by its value path
        ("/jointset/<joint>/<coordinate>/value")."""
        self.position_motion = kinematics

    def add_path_constraint(self, constraint):
        self.path_constraints.append(constraint)
        return constraint

    def create_rep(self) -> "ProblemRep":
        return ProblemRep(self)


def _vi(info: MocoVariableInfo) -> abi.mh_variable_info:
    v = abi.mh_variable_info()
    for dst, src in ((v.bounds, info.bounds), (v.initial, info.initial),
                     (v.final, info.final)):
        dst.lower, dst.upper = src.lower, src.upper
    return v


class ProblemRep:
    """MocoProblemRep: resolves default bounds and lowers to mh_problem."""

    def __init__(self, problem: MocoProblem):
        self.problem = problem
        model = problem.model
        path_eqs, bound_tables = self._path_equations(problem)
        kin = problem.position_motion
        extra = list(bound_tables)
        if kin is not None:
            qpaths = [c.path + "/value" for c in model.coordinates()]
            missing = [q for q in qpaths if q not in kin.columns]
            if missing:
                raise ValueError(f"PositionMotion: no kinematics for {missing}")
            extra.append(DataTable("__position_motion", np.asarray(kin.times, float),
                                   {q: np.asarray(kin.columns[q], float) for q in qpaths},
                                   degree=kin.degree))
        self.compiled: CompiledModel = model.compile(extra_tables=extra)
        # prescribed kinematics: coordinate values and speeds are not states
        # (MocoProblemRep.cpp:541-555)
        self.prescribed_kinematics = kin is not None
        self.state_names = [n for n in self.compiled.state_names
                            if not (self.prescribed_kinematics and
                                    (n.endswith("/value") or n.endswith("/speed")))]
        self.control_names = self.compiled.control_names
        sinfo: Dict[str, MocoVariableInfo] = {}
        cinfo: Dict[str, MocoVariableInfo] = {}
        for k, v in problem.state_infos.items():
            sinfo[k] = MocoVariableInfo(v.bounds, v.initial, v.final)
        for k, v in problem.control_infos.items():
            cinfo[k] = MocoVariableInfo(v.bounds, v.initial, v.final)
        # statebounds_ outputs: DGF normalized tendon force in [0, 5]
        # (DeGrooteFregly2016Muscle.h:131-132,304-305).
        for m in model.muscles:
            if not m.ignore_tendon_compliance:
                nm = m.path + "/normalized_tendon_force"
                info = sinfo.setdefault(nm, MocoVariableInfo())
                if not info.bounds.is_set():
                    info.bounds = MocoBounds(0.0, 5.0)
        # coordinates: range; speeds: default speed bounds (:336-362)
        for c in model.coordinates():
            vn, sn = c.path + "/value", c.path + "/speed"
            info = sinfo.setdefault(vn, MocoVariableInfo())
            if not info.bounds.is_set():
                info.bounds = MocoBounds(float(c.range[0]), float(c.range[1]))
            info = sinfo.setdefault(sn, MocoVariableInfo())
            if not info.bounds.is_set():
                info.bounds = problem.default_speed_bounds
        # controls from actuator min/max; activation from excitation (:394-427)
        for a in model.actuators:
            info = cinfo.setdefault(a.path, MocoVariableInfo())
            if not info.bounds.is_set():
                info.bounds = MocoBounds(float(a.min_control), float(a.max_control))
            if (problem.bound_activation_from_excitation and
                    isinstance(a, DeGrooteFregly2016Muscle) and
                    not a.ignore_activation_dynamics):
                an = a.path + "/activation"
                ai = sinfo.setdefault(an, MocoVariableInfo())
                if not ai.bounds.is_set():
                    ai.bounds = info.bounds
        self.state_infos = [sinfo.get(n, MocoVariableInfo()) for n in self.state_names]
        self.control_infos = [cinfo.get(n, MocoVariableInfo()) for n in self.control_names]

        # goals (endpoint-constraint mode goals become endpoint equations,
        # in goal order: MocoProblemRep::createEndpointConstraintNames)
        goals, gidx, gcol, gw = [], [], [], []
        goal_names: List[str] = []   # the mh_goal entries' goal names (objective breakdown)
        endpoint: List[abi.mh_endpoint_equation] = []
        sidx = {n: i for i, n in enumerate(self.state_names)}
        cidx = {n: i for i, n in enumerate(self.control_names)}
        self.extra_tables: List[DataTable] = []
        for g in problem.goals:
            if isinstance(g, MocoInitialActivationGoal):
                if g.mode != "endpoint_constraint":
                    raise NotImplementedError("MocoInitialActivationGoal in cost mode "
                                              "(only the endpoint-constraint default is on the "
                                              "hot path)")
                for mu in model.muscles:
                    if mu.ignore_activation_dynamics:
                        continue
                    e = abi.mh_endpoint_equation()
                    e.kind = abi.MH_ENDPOINT_INITIAL_ACTIVATION
                    e.index_a = cidx[mu.path]
                    e.index_b = sidx[mu.path + "/activation"]
                    e.g.lower, e.g.upper = 0.0, 0.0
                    endpoint.append(e)
                continue
            gs = abi.mh_goal()
            gs.weight = float(g.weight)
            gs.term_begin = len(gidx)
            gs.table = -1
            gs.exponent = 2
            if isinstance(g, MocoControlGoal):
                gs.kind = abi.MH_GOAL_CONTROL
                gs.exponent = int(g.exponent)
                if gs.exponent < 2:
                    raise ValueError("Exponent must be 2 or greater.")
                for n in self.control_names:
                    w = float(g.control_weights.get(n, 1.0))
                    if w != 0.0:
                        gidx.append(cidx[n]); gcol.append(-1); gw.append(w)
            elif isinstance(g, MocoStateTrackingGoal):
                gs.kind = abi.MH_GOAL_STATE_TRACKING
                ref = g.reference
                if ref.name not in self.compiled.table_index:
                    raise ValueError(f"reference table {ref.name} not in model")
                gs.table = self.compiled.table_index[ref.name]
                cols = self.compiled.table_columns[ref.name]
                for ci, n in enumerate(cols):
                    if n not in sidx:
                        raise ValueError(f"State reference '{n}' unrecognized.")
                    gidx.append(sidx[n]); gcol.append(ci)
                    gw.append(float(g.state_weights.get(n, 1.0)))
            elif isinstance(g, MocoFinalTimeGoal):
                gs.kind = abi.MH_GOAL_FINAL_TIME
            elif isinstance(g, MocoMarkerFinalGoal):
                if kin is not None:
                    raise NotImplementedError("MocoMarkerFinalGoal with prescribed kinematics "
                                              "(the final coordinates are not NLP states)")
                mk = model.markers.get(g.point_name)
                if mk is None:
                    raise ValueError(f"MocoMarkerFinalGoal: no point '{g.point_name}' in the model")
                body = self.compiled.body_index[mk.body]
                gs.kind = abi.MH_GOAL_MARKER_FINAL
                ref = [float(v) for v in g.reference_location]
                for ci, v in enumerate([float(v) for v in mk.location] + ref):
                    gidx.append(body); gcol.append(ci); gw.append(v)
            elif isinstance(g, ImplicitAuxiliaryDerivativesTerm):
                gs.kind = abi.MH_GOAL_AUX_DERIVATIVES
                naux = sum(1 for m in model.muscles if not m.ignore_tendon_compliance
                           and m.tendon_compliance_dynamics_mode == "implicit")
                for k in range(naux):
                    gidx.append(k); gcol.append(-1); gw.append(1.0)
            elif isinstance(g, MocoSumSquaredStateGoal):
                gs.kind = abi.MH_GOAL_SUM_SQUARED_STATE
                for n in self.state_names:
                    w = float(g.state_weights.get(n, 1.0))
                    if w != 0.0:
                        gidx.append(sidx[n]); gcol.append(-1); gw.append(w)
            else:
                raise TypeError(f"unsupported goal {type(g).__name__}")
            gs.term_count = len(gidx) - gs.term_begin
            goals.append(gs)
            goal_names.append(getattr(g, "name", "") or type(g).__name__)

        self._sinfo = (abi.mh_variable_info * max(1, len(self.state_infos)))(
            *[_vi(i) for i in self.state_infos])
        self._cinfo = (abi.mh_variable_info * max(1, len(self.control_infos)))(
            *[_vi(i) for i in self.control_infos])
        self._goals = (abi.mh_goal * max(1, len(goals)))(*goals)
        self.goal_names = goal_names
        self._gidx = np.ascontiguousarray(gidx + [0], np.int32)
        self._gcol = np.ascontiguousarray(gcol + [0], np.int32)
        self._gw = np.ascontiguousarray(gw + [0.0], float)
        p = abi.mh_problem()
        p.model = self.compiled.struct
        p.time_initial.lower, p.time_initial.upper = problem.time_initial.lower, problem.time_initial.upper
        p.time_final.lower, p.time_final.upper = problem.time_final.lower, problem.time_final.upper
        p.state_infos = self._sinfo
        p.control_infos = self._cinfo
        p.ngoals = len(goals)
        p.nterms = len(gidx)
        p.goals = self._goals
        p.goal_index = abi.iptr(self._gidx)
        p.goal_column = abi.iptr(self._gcol)
        p.goal_weight = abi.dptr(self._gw)
        for e in path_eqs:
            if e.table >= 0:   # bound table index: after the model's own
                e.table = self.compiled.table_index[bound_tables[e.table].name]
        self._path = (abi.mh_path_equation * max(1, len(path_eqs)))(*path_eqs)
        p.prescribed_kinematics = 0
        if kin is not None:
            p.prescribed_kinematics = 1
            p.kinematics_table = self.compiled.table_index["__position_motion"]
            self._kin_cols = np.arange(self.compiled.nq, dtype=np.int32)
            p.kinematics_column = abi.iptr(self._kin_cols)
        p.npath = len(path_eqs)
        p.path = self._path
        self._endpoint = (abi.mh_endpoint_equation * max(1, len(endpoint)))(*endpoint)
        p.nendpoint = len(endpoint)
        p.endpoint = self._endpoint
        p.multiplier_bounds.lower = problem.multiplier_bounds.lower
        p.multiplier_bounds.upper = problem.multiplier_bounds.upper
        p.kinematic_constraint_bounds.lower = problem.kinematic_constraint_bounds.lower
        p.kinematic_constraint_bounds.upper = problem.kinematic_constraint_bounds.upper
        # MocoParameters: bounds per parameter, one target per written property
        targets, pbounds = self._parameter_targets(problem, self.compiled)
        self.parameter_names = [par.name for par in problem.parameters]
        self._pbounds = (abi.mh_bounds * max(1, len(pbounds)))(*pbounds)
        self._ptargets = (abi.mh_parameter_target * max(1, len(targets)))(*targets)
        p.nparameters = len(pbounds)
        p.nparameter_targets = len(targets)
        p.parameter_bounds = self._pbounds
        p.parameter_targets = self._ptargets
        self.num_kinematic_constraints = len(model.constraints)
        self.num_endpoint_equations = len(endpoint)
        self.num_path_equations = len(path_eqs)
        self.struct = p
        self.num_states = len(self.state_names)
        self.num_controls = len(self.control_names)
        self.nq = self.compiled.nq
        # implicit auxiliary dynamics: DGF muscles with compliant tendons in
        # tendon_compliance_dynamics_mode "implicit" (one derivative variable
        # and one residual row per grid point each)
        self.num_aux_residuals = sum(
            1 for m in model.muscles
            if not m.ignore_tendon_compliance and m.tendon_compliance_dynamics_mode == "implicit")
        # the reference's names of the other variable blocks (MocoTrajectory
        # columns).  Multipliers: MocoProblemRep.cpp:202-230 names them
        # lambda_cid<c>_p<i> after the Simbody ConstraintIndex c, and OpenSim
        # gives every Coordinate a (disabled) lock constraint of its own
        # before the model's ConstraintSet, so the enabled couplers are
        # ConstraintIndex ncoord, ncoord + 1, ... (Rajagopal 18: 21 coordinates
        # -> lambda_cid21_p0, lambda_cid22_p0 in std_testMocoInverse_subject_
        # 18musc_solution.sto).  Slacks: the same with gamma
        # (MocoCasOCProblem.cpp:186-201).  Implicit auxiliary derivatives:
        # <component>/implicitderiv_<state> (MocoProblemRep.cpp:445-460,
        # MocoCasOCProblem.cpp:92-97), after the accelerations <coordinate>/accel
        # of implicit multibody dynamics (CasOCProblem.h:363-377).
        ncoord = len(model.coordinates())
        self.multiplier_names = [f"lambda_cid{ncoord + i}_p0" for i in range(len(model.constraints))]
        self.slack_names_all = [f"gamma_cid{ncoord + i}_p0" for i in range(len(model.constraints))]
        self.aux_derivative_names = [
            m.path + "/implicitderiv_normalized_tendon_force" for m in model.muscles
            if not m.ignore_tendon_compliance and m.tendon_compliance_dynamics_mode == "implicit"]
        self.accel_names_all = [n[:-len("speed")] + "accel" for n in self.state_names if n.endswith("/speed")]

    @staticmethod
    def _parameter_targets(problem: MocoProblem, compiled: CompiledModel):
        """MocoParameter::initializeOnModel (MocoParameter.cpp): each
        component path must name a component with the property; vector
        properties need an element in range, scalar ones none."""
        model = problem.model
        scalar = {"mass": abi.MH_PARAM_BODY_MASS, "stiffness": abi.MH_PARAM_SPRING_STIFFNESS,
                  "rest_length": abi.MH_PARAM_SPRING_REST_LENGTH, "viscosity": abi.MH_PARAM_SPRING_VISCOSITY,
                  "optimal_force": abi.MH_PARAM_ACTUATOR_OPTIMAL_FORCE,
                  "max_isometric_force": abi.MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE}
        vector = {"mass_center": (abi.MH_PARAM_BODY_MASS_CENTER, 3), "inertia": (abi.MH_PARAM_BODY_INERTIA, 6)}

        def find(path):
            key = path.rstrip("/").split("/")[-1]
            for b in model.bodies.values():
                if path in (b.name, "/bodyset/" + b.name, "/" + b.name):
                    return "body", compiled.body_index[b.name]
            for i, f in enumerate(model.springs):
                if path in (f.name, f.path) or key == f.name:
                    return "spring", i
            for i, a in enumerate(model.actuators):
                if path in (a.name, a.path):
                    return ("muscle", model.muscles.index(a)) if isinstance(a, DeGrooteFregly2016Muscle) \
                        else ("actuator", i)
            raise ValueError(f"MocoParameter: no component '{path}' in the model")
        owner = {abi.MH_PARAM_BODY_MASS: "body", abi.MH_PARAM_BODY_MASS_CENTER: "body",
                 abi.MH_PARAM_BODY_INERTIA: "body", abi.MH_PARAM_SPRING_STIFFNESS: "spring",
                 abi.MH_PARAM_SPRING_REST_LENGTH: "spring", abi.MH_PARAM_SPRING_VISCOSITY: "spring",
                 abi.MH_PARAM_ACTUATOR_OPTIMAL_FORCE: "actuator",
                 abi.MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE: "muscle"}
        targets, bounds = [], []
        names = set()
        for ip, par in enumerate(problem.parameters):
            if par.name in names:
                raise ValueError(f"MocoParameter '{par.name}': duplicate name")
            names.add(par.name)
            if not par.component_paths:
                raise ValueError(f"MocoParameter '{par.name}': no component paths")
            if par.property_name in vector:
                kind, nel = vector[par.property_name]
                if not 0 <= par.property_element < nel:
                    raise ValueError(f"MocoParameter '{par.name}': property '{par.property_name}' needs an "
                                     f"element in [0, {nel})")
                elem = par.property_element
            elif par.property_name in scalar:
                if par.property_element >= 0:
                    raise ValueError(f"MocoParameter '{par.name}': a property element was given for the "
                                     f"scalar property '{par.property_name}'")
                kind, elem = scalar[par.property_name], 0
            else:
                raise NotImplementedError(f"MocoParameter '{par.name}': property '{par.property_name}' is "
                                          "not a parameterizable property of this build")
            for path in par.component_paths:
                what, idx = find(path)
                if what != owner[kind]:
                    raise ValueError(f"MocoParameter '{par.name}': component '{path}' ({what}) has no "
                                     f"property '{par.property_name}'")
                t = abi.mh_parameter_target()
                t.parameter, t.kind, t.index, t.element = ip, kind, idx, elem
                targets.append(t)
            b = abi.mh_bounds()
            b.lower, b.upper = par.bounds.lower, par.bounds.upper
            bounds.append(b)
        return targets, bounds

    @staticmethod
    def _path_equations(problem: MocoProblem):
        """Expand path constraints to mh_path_equation rows, with the
        initializeOnModel checks of MocoControlBoundConstraint.cpp:38-118.
        Bound functions other than Constant become piecewise polynomial
        tables appended to the model's (indices into the returned list)."""
        names = problem.model.control_names()
        cidx = {n: i for i, n in enumerate(names)}
        eqs: List[abi.mh_path_equation] = []
        tables: List[DataTable] = []
        for ci, pc in enumerate(problem.path_constraints):
            if not isinstance(pc, MocoControlBoundConstraint):
                raise TypeError(f"unsupported path constraint {type(pc).__name__}")
            has_lo, has_up = pc.lower_bound is not None, pc.upper_bound is not None
            if pc.control_paths and not (has_lo or has_up):
                continue   # the reference warns and adds no equations
            for path in pc.control_paths:
                if path not in cidx:
                    raise ValueError(f"Control path '{path}' was provided but no such "
                                     "control exists in the model.")
            if pc.equality_with_lower and has_up:
                raise ValueError("If equality_with_lower==true, upper bound function "
                                 "must not be set.")
            if pc.equality_with_lower and not has_lo:
                raise ValueError("If equality_with_lower==true, lower bound function "
                                 "must be set.")
            for f in (pc.lower_bound, pc.upper_bound):
                if isinstance(f, GCVSpline):
                    lo, hi = min(f.x), max(f.x)
                    if lo > problem.time_initial.lower:
                        raise ValueError(f"The function's minimum domain value ({lo}) must be "
                                         "less than or equal to the minimum possible initial "
                                         f"time ({problem.time_initial.lower}).")
                    if hi < problem.time_final.upper:
                        raise ValueError(f"The function's maximum domain value ({hi}) must be "
                                         "greater than or equal to the maximum possible final "
                                         f"time ({problem.time_final.upper}).")

            def bound_ref(f, which):
                pp = f.ppoly()
                if pp is None:
                    return -1, 0, float(f.value)
                name = f"__path{ci}_{which}"
                if not any(t.name == name for t in tables):
                    br, cf = pp
                    tables.append(DataTable(name=name, times=np.asarray(br, float),
                                            columns={"bound": np.zeros(len(br))},
                                            ppoly=(np.asarray(br, float), np.asarray(cf, float))))
                return [t.name for t in tables].index(name), 0, 0.0

            for path in pc.control_paths:
                for which, f in (("lower", pc.lower_bound), ("upper", pc.upper_bound)):
                    if f is None:
                        continue
                    e = abi.mh_path_equation()
                    e.kind = abi.MH_PATH_CONTROL_BOUND
                    e.index = cidx[path]
                    e.table, e.column, e.value = bound_ref(f, which)
                    if pc.equality_with_lower:
                        e.g.lower, e.g.upper = 0.0, 0.0
                    elif which == "lower":
                        e.g.lower, e.g.upper = 0.0, math.inf
                    else:
                        e.g.lower, e.g.upper = -math.inf, 0.0
                    eqs.append(e)
        return eqs, tables
