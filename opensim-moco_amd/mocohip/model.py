"""Host-side model compiler: OpenSim-like model objects -> mh_model tape.

This mirrors the parts of OpenSim's Model that the collocation hot path
reads (bodies/joints/coordinates, DeGrooteFregly2016 muscles with their
GeometryPath, CoordinateActuators, ExternalForces) and lowers them to the
plain C structs of include/mocohip.h.

Ordering rules restated from the reference:
  * generalized coordinates follow Simbody's mobilized-body order, which
    OpenSim's MultibodyGraphMaker grows one tree level at a time (joints in
    model order within a level) -- pinned by the column order of
    Moco/Tests/std_testMocoTrackGait10dof18musc_solution.sto:14;
  * auxiliary states per muscle: activation, then normalized tendon force
    (DeGrooteFregly2016Muscle.cpp:151-164); muscles in force-set order;
  * controls: actuators in component order (MocoUtilities.cpp:557-587).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .splines import gcv_interpolating_ppoly


# --------------------------------------------------------------------------
# Functions of one coordinate.
# --------------------------------------------------------------------------
@dataclass
class Function:
    kind: int
    coord: Optional[str] = None
    a: float = 0.0
    b: float = 0.0
    scale: float = 1.0
    x: Sequence[float] = ()
    y: Sequence[float] = ()

    @staticmethod
    def constant(v: float) -> "Function":
        return Function(abi.MH_FN_CONSTANT, None, a=float(v))

    @staticmethod
    def linear(coord: str, slope: float = 1.0, intercept: float = 0.0,
               scale: float = 1.0) -> "Function":
        return Function(abi.MH_FN_LINEAR, coord, a=float(slope),
                        b=float(intercept), scale=float(scale))

    @staticmethod
    def simm_spline(coord: str, x, y, scale: float = 1.0) -> "Function":
        return Function(abi.MH_FN_SIMMSPLINE, coord, x=list(map(float, x)),
                        y=list(map(float, y)), scale=float(scale))

    def scaled(self, s: float) -> "Function":
        """MultiplierFunction."""
        if self.kind == abi.MH_FN_CONSTANT:
            return Function.constant(self.a * s)
        f = Function(self.kind, self.coord, self.a, self.b, self.scale * s,
                     self.x, self.y)
        return f


# --------------------------------------------------------------------------
# Frames / rotations.
# --------------------------------------------------------------------------
def rot_x(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]], float)


def rot_y(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], float)


def rot_z(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], float)


def _mm3(A, B):
    """3x3 product with each entry summed left to right (no BLAS): the same
    IEEE operations as the C++ builder (csrc/host/mh_builder.cpp mm3)."""
    return [[(A[i][0] * B[0][j] + A[i][1] * B[1][j]) + A[i][2] * B[2][j] for j in range(3)]
            for i in range(3)]


def body_fixed_xyz(angles) -> np.ndarray:
    """OpenSim frame orientation: Euler XYZ body-fixed angles,
    rot_x(a0) rot_y(a1) rot_z(a2)."""
    X, Y, Z = (r(float(a)).tolist() for r, a in zip((rot_x, rot_y, rot_z), angles))
    return np.array(_mm3(_mm3(X, Y), Z), float)


def unit3(d) -> List[float]:
    """d / |d| with |d| = sqrt((d0 d0 + d1 d1) + d2 d2) (as the C++ builder)."""
    d0, d1, d2 = (float(v) for v in d)
    n = math.sqrt(d0 * d0 + d1 * d1 + d2 * d2)
    return [d0 / n, d1 / n, d2 / n]


@dataclass
class Body:
    name: str
    mass: float
    com: Sequence[float] = (0.0, 0.0, 0.0)
    inertia: Sequence[float] = (0, 0, 0, 0, 0, 0)   # xx yy zz xy xz yz


@dataclass
class Coordinate:
    name: str
    range: Sequence[float] = (-math.inf, math.inf)
    motion_type: str = "rotational"
    default_value: float = 0.0
    path: str = ""        # OpenSim absolute path, e.g. /jointset/j/q


@dataclass
class Axis:
    type: int            # abi.MH_AXIS_ROTATION / TRANSLATION
    dir: Sequence[float]
    func: Function


@dataclass
class Joint:
    name: str
    parent: str          # body name or "ground"
    child: str
    coordinates: List[Coordinate]
    axes: List[Axis]
    loc_in_parent: Sequence[float] = (0, 0, 0)
    orient_in_parent: Sequence[float] = (0, 0, 0)
    loc_in_child: Sequence[float] = (0, 0, 0)
    orient_in_child: Sequence[float] = (0, 0, 0)

    @staticmethod
    def pin(name, parent, child, coord: Coordinate, **frames) -> "Joint":
        """PinJoint: rotation about z of the joint frame."""
        return Joint(name, parent, child, [coord],
                     [Axis(abi.MH_AXIS_ROTATION, (0, 0, 1),
                           Function.linear(coord.name))], **frames)

    @staticmethod
    def slider(name, parent, child, coord: Coordinate, **frames) -> "Joint":
        """SliderJoint: translation along x of the joint frame."""
        return Joint(name, parent, child, [coord],
                     [Axis(abi.MH_AXIS_TRANSLATION, (1, 0, 0),
                           Function.linear(coord.name))], **frames)

    @staticmethod
    def planar(name, parent, child, rz: Coordinate, tx: Coordinate,
               ty: Coordinate, **frames) -> "Joint":
        """PlanarJoint: rotation about z, translation along x and y."""
        return Joint(name, parent, child, [rz, tx, ty], [
            Axis(abi.MH_AXIS_ROTATION, (0, 0, 1), Function.linear(rz.name)),
            Axis(abi.MH_AXIS_TRANSLATION, (1, 0, 0), Function.linear(tx.name)),
            Axis(abi.MH_AXIS_TRANSLATION, (0, 1, 0), Function.linear(ty.name)),
        ], **frames)

    @staticmethod
    def weld(name, parent, child, **frames) -> "Joint":
        return Joint(name, parent, child, [], [], **frames)


@dataclass
class PathPoint:
    body: str
    loc: Sequence[float]
    kind: int = abi.MH_PP_FIXED
    coord: Optional[str] = None         # conditional
    range: Sequence[float] = (0.0, 0.0)
    fx: Optional[Function] = None       # moving
    fy: Optional[Function] = None
    fz: Optional[Function] = None
    name: str = ""


@dataclass
class DeGrooteFregly2016Muscle:
    """Properties and defaults of DeGrooteFregly2016Muscle
    (DeGrooteFregly2016Muscle.cpp:52-63)."""
    name: str
    points: List[PathPoint]
    max_isometric_force: float = 1000.0
    optimal_fiber_length: float = 0.1
    tendon_slack_length: float = 0.2
    pennation_angle_at_optimal: float = 0.0
    max_contraction_velocity: float = 10.0
    activation_time_constant: float = 0.015
    deactivation_time_constant: float = 0.060
    default_activation: float = 0.5
    default_normalized_tendon_force: float = 0.5
    active_force_width_scale: float = 1.0
    fiber_damping: float = 0.0
    passive_fiber_strain_at_one_norm_force: float = 0.6
    tendon_strain_at_one_norm_force: float = 0.049
    ignore_passive_fiber_force: bool = False
    ignore_activation_dynamics: bool = False
    ignore_tendon_compliance: bool = False
    tendon_compliance_dynamics_mode: str = "explicit"
    min_control: float = 0.0
    max_control: float = 1.0
    path: str = ""
    # GeometryPath PathWrapSet, in order: (wrap object name, range begin,
    # range end) with OpenSim's 1-based point range (< 1: first / last)
    path_wraps: List[tuple] = field(default_factory=list)


@dataclass
class WrapCylinder:
    """OpenSim WrapCylinder in a body's WrapObjectSet: axis = the z axis of
    its frame, which is rotated by the body-fixed X-Y-Z sequence
    ``xyz_body_rotation`` and translated by ``translation`` in the body;
    ``quadrant`` "all" / "+x" / "-x" / "+y" / "-y" (include/mocohip.h
    mh_wrap_object)."""
    name: str
    body: str
    radius: float
    length: float = 1.0
    xyz_body_rotation: Sequence[float] = (0.0, 0.0, 0.0)
    translation: Sequence[float] = (0.0, 0.0, 0.0)
    quadrant: str = "all"
    active: bool = True


def quadrant_axis_sign(quadrant: str):
    """WrapObject quadrant -> (wrap axis, wrap sign); "all" -> (0, 0)."""
    q = quadrant.strip().lower()
    if q in ("all", ""):
        return 0, 0
    sign = -1 if q.startswith("-") else 1
    ax = q.lstrip("+-")
    if ax not in ("x", "y", "z"):
        raise ValueError(f"bad wrap quadrant {quadrant!r}")
    if ax == "z":
        raise NotImplementedError("WrapCylinder quadrant along its axis")
    return "xy".index(ax), sign


@dataclass
class CoordinateActuator:
    name: str
    coordinate: str
    optimal_force: float = 1.0
    min_control: float = -math.inf
    max_control: float = math.inf
    path: str = ""


@dataclass
class SpringGeneralizedForce:
    """OpenSim SpringGeneralizedForce (opensim-core, third-party): the
    generalized force -stiffness (q - rest_length) - viscosity u on one
    coordinate (include/mocohip.h mh_spring; testMocoParameters.cpp:52-57);
    path /forceset/<name>."""
    name: str
    coordinate: str
    stiffness: float = 0.0
    rest_length: float = 0.0
    viscosity: float = 0.0
    path: str = ""


@dataclass
class Marker:
    """OpenSim::Marker: a point fixed on a body (``location`` in the body
    frame); path /markerset/<name>."""
    name: str
    body: str                # body name or "ground"
    location: Sequence[float] = (0.0, 0.0, 0.0)
    path: str = ""


@dataclass
class DataTable:
    """Time series; splined with the GCVSpline restatement (splines.py)."""
    name: str
    times: np.ndarray
    columns: Dict[str, np.ndarray]
    degree: int = 3
    # explicit piecewise polynomial (breaks[nseg+1], coefs[nseg, ncol,
    # degree+1]) instead of splining the samples (path-constraint bounds)
    ppoly: Optional[tuple] = None


@dataclass
class ExternalForce:
    name: str
    body: str
    table: str
    force_identifier: Optional[str] = None     # e.g. "ground_force_v"
    point_identifier: Optional[str] = None
    torque_identifier: Optional[str] = None


@dataclass
class CoordinateCouplerConstraint:
    """OpenSim CoordinateCouplerConstraint with one independent coordinate:
    q[dependent] = scale_factor * function(q[independent]) (the Simbody
    CoordinateCoupler of OpenSim's CompoundFunction; include/mocohip.h
    mh_constraint).  ``function.coord`` names the independent coordinate."""
    name: str
    dependent: str
    function: Function
    scale_factor: float = 1.0


class Model:
    def __init__(self, name: str = "model", gravity=(0, -9.80665, 0)):
        self.name = name
        self.gravity = tuple(float(g) for g in gravity)
        self.bodies: Dict[str, Body] = {}
        self.joints: List[Joint] = []
        self.muscles: List[DeGrooteFregly2016Muscle] = []
        self.actuators: List[object] = []       # force-set order
        self.tables: Dict[str, DataTable] = {}
        self.external_forces: List[ExternalForce] = []
        self.markers: Dict[str, Marker] = {}    # by path
        self.constraints: List[CoordinateCouplerConstraint] = []   # enabled ones
        self.wraps: Dict[str, WrapCylinder] = {}
        self.springs: List[SpringGeneralizedForce] = []

    # building ---------------------------------------------------------------
    def add_body(self, body: Body):
        self.bodies[body.name] = body
        return body

    def add_joint(self, joint: Joint):
        for c in joint.coordinates:
            if not c.path:
                c.path = f"/jointset/{joint.name}/{c.name}"
        self.joints.append(joint)
        return joint

    def add_muscle(self, m: DeGrooteFregly2016Muscle):
        if not m.path:
            m.path = f"/forceset/{m.name}"
        self.muscles.append(m)
        self.actuators.append(m)
        return m

    def add_coordinate_actuator(self, a: CoordinateActuator):
        if not a.path:
            a.path = f"/forceset/{a.name}"
        self.actuators.append(a)
        return a

    def add_spring(self, f: SpringGeneralizedForce):
        if not f.path:
            f.path = f"/forceset/{f.name}"
        self.springs.append(f)
        return f

    def add_table(self, t: DataTable):
        self.tables[t.name] = t
        return t

    def add_external_force(self, e: ExternalForce):
        self.external_forces.append(e)
        return e

    def add_constraint(self, k: CoordinateCouplerConstraint):
        self.constraints.append(k)
        return k

    def add_wrap(self, w: WrapCylinder):
        self.wraps[w.name] = w
        return w

    def replace_joints_with_welds(self, names: Sequence[str]):
        """ModOpReplaceJointsWithWelds (ModelFactory::replaceJointWithWeldJoint,
        Moco/Moco/ModelOperators.h, ModelFactory.cpp): each named joint becomes
        a WeldJoint with the same parent / child frames; its coordinates, and
        the actuators on them, are removed."""
        gone = set()
        for j in self.joints:
            if j.name in names:
                gone.update(c.name for c in j.coordinates)
                j.coordinates = []
                j.axes = []
        missing = set(names) - {j.name for j in self.joints}
        if missing:
            raise ValueError(f"no joints {sorted(missing)}")
        for m in self.muscles:
            for p in m.points:
                for f in (p.fx, p.fy, p.fz):
                    if f is not None and f.coord in gone:
                        raise NotImplementedError(f"{m.name}: moving point on welded {f.coord}")
                if p.coord in gone:
                    raise NotImplementedError(f"{m.name}: conditional point on welded {p.coord}")
        self.actuators = [a for a in self.actuators
                          if not (isinstance(a, CoordinateActuator) and a.coordinate in gone)]

    def add_marker(self, mk: Marker):
        if not mk.path:
            mk.path = f"/markerset/{mk.name}"
        self.markers[mk.path] = mk
        return mk

    # ordering ---------------------------------------------------------------
    def tree_order(self) -> List[Joint]:
        """Joints in Simbody mobilized-body order: breadth-first by tree
        level, model joint order within a level (MultibodyGraphMaker)."""
        order: List[Joint] = []
        placed = {"ground"}
        remaining = list(self.joints)
        while remaining:
            level = [j for j in remaining if j.parent in placed]
            if not level:
                raise ValueError("model graph is not a tree rooted at ground")
            for j in level:
                order.append(j)
            for j in level:
                placed.add(j.child)
            remaining = [j for j in remaining if j not in level]
        return order

    def coordinates(self) -> List[Coordinate]:
        return [c for j in self.tree_order() for c in j.coordinates]

    def coordinate_index(self) -> Dict[str, int]:
        return {c.name: i for i, c in enumerate(self.coordinates())}

    def state_names(self) -> List[str]:
        qs = self.coordinates()
        names = [c.path + "/value" for c in qs] + [c.path + "/speed" for c in qs]
        for m in self.muscles:
            if not m.ignore_activation_dynamics:
                names.append(m.path + "/activation")
            if not m.ignore_tendon_compliance:
                names.append(m.path + "/normalized_tendon_force")
        return names

    def control_names(self) -> List[str]:
        return [a.path for a in self.actuators]

    # lowering ---------------------------------------------------------------
    def compile(self, extra_tables: Sequence[DataTable] = ()) -> "CompiledModel":
        """Lower to mh_model.  ``extra_tables`` (problem-level functions of
        time, e.g. path-constraint bounds) are appended after the model's
        own tables, which keep their indices."""
        return CompiledModel(self, extra_tables)


def _arr(struct_type, items):
    n = len(items)
    arr = (struct_type * max(n, 1))()
    for i, it in enumerate(items):
        arr[i] = it
    return arr


class CompiledModel:
    """Owns the C arrays that back an mh_model."""

    def __init__(self, model: Model, extra_tables: Sequence[DataTable] = ()):
        self.model = model
        qidx = model.coordinate_index()
        self.qidx = qidx
        joints = model.tree_order()
        body_index = {"ground": -1}
        for i, j in enumerate(joints):
            body_index[j.child] = i
        self.body_index = body_index
        funcs: List[abi.mh_function] = []
        knot_x: List[float] = []
        knot_y: List[float] = []

        def add_function(f: Optional[Function]) -> int:
            if f is None:
                return -1
            fs = abi.mh_function()
            fs.kind = f.kind
            fs.coord = qidx[f.coord] if f.coord is not None and f.kind != abi.MH_FN_CONSTANT else -1
            fs.a, fs.b, fs.scale = f.a, f.b, f.scale
            if f.kind == abi.MH_FN_SIMMSPLINE:
                fs.knot_begin = len(knot_x)
                fs.knot_count = len(f.x)
                knot_x.extend(f.x)
                knot_y.extend(f.y)
            funcs.append(fs)
            return len(funcs) - 1

        bodies, axes = [], []
        for j in joints:
            B = model.bodies[j.child]
            b = abi.mh_body()
            b.parent = body_index[j.parent]
            b.mass = B.mass
            b.com[:] = list(map(float, B.com))
            b.inertia[:] = list(map(float, B.inertia))
            R_PF = body_fixed_xyz(j.orient_in_parent)
            R_BM = body_fixed_xyz(j.orient_in_child)
            b.R_PF[:] = R_PF.reshape(-1).tolist()
            b.p_PF[:] = list(map(float, j.loc_in_parent))
            b.R_BM[:] = R_BM.reshape(-1).tolist()
            b.p_BM[:] = list(map(float, j.loc_in_child))
            b.axis_begin = len(axes)
            for ax in j.axes:
                a = abi.mh_axis()
                a.type = ax.type
                a.dir[:] = unit3(ax.dir)
                a.func = add_function(ax.func)
                axes.append(a)
            b.axis_count = len(axes) - b.axis_begin
            bodies.append(b)

        points, muscles = [], []
        for m in model.muscles:
            ms = abi.mh_muscle()
            ms.point_begin = len(points)
            for p in m.points:
                ps = abi.mh_path_point()
                ps.kind = p.kind
                ps.body = body_index[p.body]
                ps.loc[:] = list(map(float, p.loc))
                ps.coord = qidx[p.coord] if p.coord is not None else -1
                ps.range[:] = list(map(float, p.range))
                ps.fx = add_function(p.fx)
                ps.fy = add_function(p.fy)
                ps.fz = add_function(p.fz)
                points.append(ps)
            ms.point_count = len(points) - ms.point_begin
            ms.ignore_activation_dynamics = int(m.ignore_activation_dynamics)
            ms.ignore_tendon_compliance = int(m.ignore_tendon_compliance)
            ms.ignore_passive_fiber_force = int(m.ignore_passive_fiber_force)
            ms.tendon_dynamics_implicit = int(
                m.tendon_compliance_dynamics_mode == "implicit")
            for k in ("max_isometric_force", "optimal_fiber_length",
                      "tendon_slack_length", "pennation_angle_at_optimal",
                      "max_contraction_velocity", "activation_time_constant",
                      "deactivation_time_constant", "fiber_damping",
                      "passive_fiber_strain_at_one_norm_force",
                      "tendon_strain_at_one_norm_force",
                      "active_force_width_scale"):
                setattr(ms, k, float(getattr(m, k)))
            muscles.append(ms)

        # wrap surfaces (in model order) and the PathWrap list per muscle
        wraps, pathwraps = [], []
        wrap_index = {}
        for w in model.wraps.values():
            if not w.active:
                continue
            ws = abi.mh_wrap_object()
            ws.kind = abi.MH_WRAP_CYLINDER
            ws.body = body_index[w.body]
            ws.wrap_axis, ws.wrap_sign = quadrant_axis_sign(w.quadrant)
            ws.R_BW[:] = body_fixed_xyz(w.xyz_body_rotation).reshape(-1).tolist()
            ws.p_BW[:] = list(map(float, w.translation))
            ws.radius = float(w.radius)
            ws.length = float(w.length)
            wrap_index[w.name] = len(wraps)
            wraps.append(ws)
        for im, m in enumerate(model.muscles):
            for (wname, r0, r1) in m.path_wraps:
                if wname not in wrap_index:
                    if wname in model.wraps:
                        continue        # inactive wrap object
                    raise ValueError(f"{m.name}: unknown wrap object {wname}")
                pw = abi.mh_path_wrap()
                pw.muscle, pw.wrap = im, wrap_index[wname]
                pw.range_begin, pw.range_end = int(r0), int(r1)
                pathwraps.append(pw)
        self._wraps = _arr(abi.mh_wrap_object, wraps)
        self._pathwraps = _arr(abi.mh_path_wrap, pathwraps)

        muscle_index = {id(m): i for i, m in enumerate(model.muscles)}
        acts = []
        for a in model.actuators:
            s = abi.mh_actuator()
            if isinstance(a, DeGrooteFregly2016Muscle):
                s.kind = abi.MH_ACT_MUSCLE
                s.target = muscle_index[id(a)]
                s.optimal_force = 1.0
            else:
                s.kind = abi.MH_ACT_COORDINATE
                s.target = qidx[a.coordinate]
                s.optimal_force = float(a.optimal_force)
            acts.append(s)

        # data tables -> piecewise polynomials
        tables, breaks, coefs = [], [], []
        self.table_index: Dict[str, int] = {}
        self.table_columns: Dict[str, List[str]] = {}
        all_tables = list(model.tables.items()) + [(t.name, t) for t in extra_tables]
        for name, t in all_tables:
            cols = list(t.columns.keys())
            if t.ppoly is not None:
                br, cf = t.ppoly
            else:
                br, cf = gcv_interpolating_ppoly(
                    np.asarray(t.times, float),
                    np.stack([np.asarray(t.columns[c], float) for c in cols], 1),
                    t.degree)
            ts = abi.mh_table()
            ts.nseg = len(br) - 1
            ts.degree = cf.shape[-1] - 1
            ts.ncol = len(cols)
            ts.break_begin = len(breaks)
            ts.coef_begin = len(coefs)
            breaks.extend(br.tolist())
            coefs.extend(cf.reshape(-1).tolist())
            self.table_index[name] = len(tables)
            self.table_columns[name] = cols
            tables.append(ts)

        ext = []
        for e in model.external_forces:
            es = abi.mh_external_force()
            es.body = body_index[e.body]
            es.table = self.table_index[e.table]
            cols = self.table_columns[e.table]

            def col3(ident):
                if ident is None:
                    return -1
                i = cols.index(ident + "x")
                assert cols[i + 1] == ident + "y" and cols[i + 2] == ident + "z"
                return i
            es.force_col = col3(e.force_identifier)
            es.point_col = col3(e.point_identifier)
            es.torque_col = col3(e.torque_identifier)
            ext.append(es)

        self._bodies = _arr(abi.mh_body, bodies)
        self._axes = _arr(abi.mh_axis, axes)
        self._funcs = _arr(abi.mh_function, funcs)
        self._kx = np.ascontiguousarray(knot_x + [0.0], float)
        self._ky = np.ascontiguousarray(knot_y + [0.0], float)
        self._muscles = _arr(abi.mh_muscle, muscles)
        self._points = _arr(abi.mh_path_point, points)
        self._acts = _arr(abi.mh_actuator, acts)
        self._tables = _arr(abi.mh_table, tables)
        self._breaks = np.ascontiguousarray(breaks + [0.0], float)
        self._coefs = np.ascontiguousarray(coefs + [0.0], float)
        self._ext = _arr(abi.mh_external_force, ext)
        # kinematic constraints: their functions after every other function
        # (models without constraints keep their function list and hash)
        kcs = []
        for k in model.constraints:
            if k.function.kind == abi.MH_FN_CONSTANT or k.function.coord is None:
                raise ValueError(f"constraint {k.name}: needs a function of the independent coordinate")
            ks = abi.mh_constraint()
            ks.kind = abi.MH_KC_COORDINATE_COUPLER
            ks.dependent = qidx[k.dependent]
            ks.func = add_function(k.function)
            ks.scale = float(k.scale_factor)
            kcs.append(ks)
        self._funcs = _arr(abi.mh_function, funcs)
        self._kx = np.ascontiguousarray(knot_x + [0.0], float)
        self._ky = np.ascontiguousarray(knot_y + [0.0], float)
        self._kcs = _arr(abi.mh_constraint, kcs)
        springs = []
        for f in model.springs:
            ss = abi.mh_spring()
            ss.coord = qidx[f.coordinate]
            ss.stiffness, ss.rest_length, ss.viscosity = float(f.stiffness), float(f.rest_length), float(f.viscosity)
            springs.append(ss)
        self._springs = _arr(abi.mh_spring, springs)

        mm = abi.mh_model()
        mm.nq = len(qidx)
        mm.nbodies = len(bodies)
        mm.naxes = len(axes)
        mm.nfunctions = len(funcs)
        mm.nknots = len(knot_x)
        mm.nconstraints = len(kcs)
        mm.constraints = self._kcs
        mm.nmuscles = len(muscles)
        mm.npoints = len(points)
        mm.nactuators = len(acts)
        mm.ntables = len(tables)
        mm.nbreaks = len(breaks)
        mm.ncoefs = len(coefs)
        mm.nexternal = len(ext)
        mm.gravity[:] = list(model.gravity)
        mm.bodies = self._bodies
        mm.axes = self._axes
        mm.functions = self._funcs
        mm.knot_x = abi.dptr(self._kx)
        mm.knot_y = abi.dptr(self._ky)
        mm.muscles = self._muscles
        mm.points = self._points
        mm.actuators = self._acts
        mm.tables = self._tables
        mm.table_breaks = abi.dptr(self._breaks)
        mm.table_coefs = abi.dptr(self._coefs)
        mm.external = self._ext
        mm.nwraps = len(wraps)
        mm.npathwraps = len(pathwraps)
        mm.wraps = self._wraps
        mm.pathwraps = self._pathwraps
        mm.nsprings = len(springs)
        mm.springs = self._springs
        self.struct = mm
        self.nq = mm.nq
        self.state_names = model.state_names()
        self.control_names = model.control_names()


# --------------------------------------------------------------------------
# JSON round trip (committed model data under mocohip/data/).
# --------------------------------------------------------------------------
def _fn_to(f: Optional[Function]):
    if f is None:
        return None
    return {"kind": f.kind, "coord": f.coord, "a": f.a, "b": f.b,
            "scale": f.scale, "x": list(f.x), "y": list(f.y)}


def _fn_from(d) -> Optional[Function]:
    if d is None:
        return None
    return Function(d["kind"], d["coord"], d["a"], d["b"], d["scale"],
                    d["x"], d["y"])


def model_to_dict(m: Model) -> dict:
    return {
        "name": m.name, "gravity": list(m.gravity),
        "bodies": [{"name": b.name, "mass": b.mass, "com": list(b.com),
                    "inertia": list(b.inertia)} for b in m.bodies.values()],
        "joints": [{
            "name": j.name, "parent": j.parent, "child": j.child,
            "coordinates": [{"name": c.name, "range": list(c.range),
                             "motion_type": c.motion_type,
                             "default_value": c.default_value, "path": c.path}
                            for c in j.coordinates],
            "axes": [{"type": a.type, "dir": list(a.dir), "func": _fn_to(a.func)}
                     for a in j.axes],
            "loc_in_parent": list(j.loc_in_parent),
            "orient_in_parent": list(j.orient_in_parent),
            "loc_in_child": list(j.loc_in_child),
            "orient_in_child": list(j.orient_in_child)} for j in m.joints],
        "actuators": [
            ({"type": "muscle", **{k: getattr(a, k) for k in a.__dataclass_fields__
                                    if k != "points"},
              "points": [{"body": p.body, "loc": list(p.loc), "kind": p.kind,
                          "coord": p.coord, "range": list(p.range),
                          "fx": _fn_to(p.fx), "fy": _fn_to(p.fy),
                          "fz": _fn_to(p.fz), "name": p.name} for p in a.points]}
             if isinstance(a, DeGrooteFregly2016Muscle) else
             {"type": "coordinate_actuator", "name": a.name,
              "coordinate": a.coordinate, "optimal_force": a.optimal_force,
              "min_control": a.min_control, "max_control": a.max_control,
              "path": a.path})
            for a in m.actuators],
        "markers": [{"name": k.name, "body": k.body, "location": list(k.location), "path": k.path}
                    for k in m.markers.values()],
        "wraps": [{"name": w.name, "body": w.body, "radius": w.radius, "length": w.length,
                   "xyz_body_rotation": list(w.xyz_body_rotation),
                   "translation": list(w.translation), "quadrant": w.quadrant,
                   "active": w.active} for w in m.wraps.values()],
        "constraints": [{"name": k.name, "dependent": k.dependent, "function": _fn_to(k.function),
                         "scale_factor": k.scale_factor} for k in m.constraints],
        "springs": [{"name": f.name, "coordinate": f.coordinate, "stiffness": f.stiffness,
                     "rest_length": f.rest_length, "viscosity": f.viscosity, "path": f.path}
                    for f in m.springs],
    }


def model_from_dict(d: dict) -> Model:
    m = Model(d["name"], tuple(d["gravity"]))
    for b in d["bodies"]:
        m.add_body(Body(b["name"], b["mass"], tuple(b["com"]), tuple(b["inertia"])))
    for j in d["joints"]:
        coords = [Coordinate(c["name"], tuple(c["range"]), c["motion_type"],
                             c["default_value"], c["path"]) for c in j["coordinates"]]
        axes = [Axis(a["type"], tuple(a["dir"]), _fn_from(a["func"])) for a in j["axes"]]
        m.add_joint(Joint(j["name"], j["parent"], j["child"], coords, axes,
                          tuple(j["loc_in_parent"]), tuple(j["orient_in_parent"]),
                          tuple(j["loc_in_child"]), tuple(j["orient_in_child"])))
    for a in d["actuators"]:
        if a["type"] == "muscle":
            pts = [PathPoint(p["body"], tuple(p["loc"]), p["kind"], p["coord"],
                             tuple(p["range"]), _fn_from(p["fx"]), _fn_from(p["fy"]),
                             _fn_from(p["fz"]), p["name"]) for p in a["points"]]
            kw = {k: v for k, v in a.items() if k not in ("type", "points")}
            kw["path_wraps"] = [tuple(w) for w in kw.get("path_wraps", [])]
            m.add_muscle(DeGrooteFregly2016Muscle(points=pts, **kw))
        else:
            m.add_coordinate_actuator(CoordinateActuator(
                a["name"], a["coordinate"], a["optimal_force"], a["min_control"],
                a["max_control"], a["path"]))
    for k in d.get("markers", []):
        m.add_marker(Marker(k["name"], k["body"], tuple(k["location"]), k.get("path", "")))
    for w in d.get("wraps", []):
        m.add_wrap(WrapCylinder(w["name"], w["body"], w["radius"], w["length"],
                                tuple(w["xyz_body_rotation"]), tuple(w["translation"]),
                                w["quadrant"], w["active"]))
    for k in d.get("constraints", []):
        m.add_constraint(CoordinateCouplerConstraint(k["name"], k["dependent"],
                                                     _fn_from(k["function"]), k["scale_factor"]))
    for f in d.get("springs", []):
        m.add_spring(SpringGeneralizedForce(f["name"], f["coordinate"], f["stiffness"], f["rest_length"],
                                            f["viscosity"], f.get("path", "")))
    return m
