"""OpenSim .osim reader (model-compiler front end).

Reads the subset of OpenSim 3.x (Version 30000, joints nested in bodies) and
4.x (JointSet with offset frames) XML that the collocation hot path needs:
bodies, Pin/Slider/Planar/Weld/CustomJoint with Constant / LinearFunction /
SimmSpline / MultiplierFunction transform axes, muscles with PathPoint /
ConditionalPathPoint / MovingPathPoint geometry, CoordinateActuators.

Muscles are converted to DeGrooteFregly2016Muscle exactly as
DeGrooteFregly2016Muscle::replaceMuscles does
(Moco/Moco/Components/DeGrooteFregly2016Muscle.cpp:933-1054).  Property
defaults of Millard2012EquilibriumMuscle / Thelen2003Muscle that are not
written in a file are opensim-core defaults, restated (third-party).
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

from . import abi
from .model import (Axis, Body, Coordinate, CoordinateActuator,
                    CoordinateCouplerConstraint, DeGrooteFregly2016Muscle,
                    Function, Joint, Model, PathPoint, WrapCylinder)

# opensim-core Millard2012EquilibriumMuscle defaults (restated).
MILLARD_DEFAULTS = dict(fiber_damping=0.1, default_activation=0.05,
                        activation_time_constant=0.01,
                        deactivation_time_constant=0.04,
                        passive_strain=0.7, tendon_strain=0.049)


def _floats(text: Optional[str]) -> List[float]:
    return [float(v) for v in (text or "").split()]


def _child(el, tag):
    return el.find(tag) if el is not None else None


def _text(el, tag, default=None):
    c = _child(el, tag)
    return c.text.strip() if c is not None and c.text is not None else default


def _float(el, tag, default=None):
    t = _text(el, tag)
    return float(t) if t is not None and t != "" else default


def _bool(el, tag, default=False):
    t = _text(el, tag)
    return default if t is None else t.strip().lower() == "true"


FUNCTION_TAGS = ("Constant", "LinearFunction", "SimmSpline", "MultiplierFunction",
                 "PiecewiseLinearFunction", "NaturalCubicSpline", "GCVSpline", "PolynomialFunction")


def parse_function(fel, coord: Optional[str]) -> Function:
    """Parse the single function element below ``fel``."""
    if fel is None:
        return Function.constant(0.0)
    kids = list(fel)
    f = kids[0] if fel.tag in ("function", "x_location", "y_location",
                               "z_location", "coupled_coordinates_function") else fel
    tag = f.tag
    if tag == "Constant":
        return Function.constant(_float(f, "value", 0.0))
    if tag == "LinearFunction":
        co = _floats(_text(f, "coefficients", "1 0"))
        return Function.linear(coord, co[0], co[1])
    if tag == "SimmSpline":
        return Function.simm_spline(coord, _floats(_text(f, "x")), _floats(_text(f, "y")))
    if tag == "MultiplierFunction":
        inner = parse_function(_child(f, "function"), coord)
        return inner.scaled(_float(f, "scale", 1.0))
    raise NotImplementedError(f"OpenSim function {tag} not supported")


def _coordinates(jel) -> List[Coordinate]:
    out = []
    cs = jel.find("CoordinateSet/objects")
    if cs is None:
        cs = jel.find("coordinates")
    if cs is None:
        return out
    for c in cs.findall("Coordinate"):
        rng = _floats(_text(c, "range", "-inf inf")) or [-math.inf, math.inf]
        out.append(Coordinate(c.get("name"), tuple(rng),
                              _text(c, "motion_type", "rotational"),
                              _float(c, "default_value", 0.0)))
    return out


def _axes_for(jel, jtype: str, coords: List[Coordinate]) -> List[Axis]:
    if jtype == "PinJoint":
        return [Axis(abi.MH_AXIS_ROTATION, (0, 0, 1), Function.linear(coords[0].name))]
    if jtype == "SliderJoint":
        return [Axis(abi.MH_AXIS_TRANSLATION, (1, 0, 0), Function.linear(coords[0].name))]
    if jtype == "PlanarJoint":
        return [Axis(abi.MH_AXIS_ROTATION, (0, 0, 1), Function.linear(coords[0].name)),
                Axis(abi.MH_AXIS_TRANSLATION, (1, 0, 0), Function.linear(coords[1].name)),
                Axis(abi.MH_AXIS_TRANSLATION, (0, 1, 0), Function.linear(coords[2].name))]
    if jtype == "WeldJoint":
        return []
    if jtype == "CustomJoint":
        st = jel.find("SpatialTransform")
        axes = []
        rot, trans = [], []
        for ta in st.findall("TransformAxis"):
            name = ta.get("name")
            cn = (_text(ta, "coordinates", "") or "").split()
            if len(cn) > 1:
                raise NotImplementedError("TransformAxis with >1 coordinate")
            coord = cn[0] if cn else None
            # OpenSim 3: <function><Kind/></function>; OpenSim 4: <Kind name="function"/>
            fel = ta.find("function")
            if fel is None:
                fel = next((ch for ch in ta if ch.tag in FUNCTION_TAGS), None)
            fn = parse_function(fel, coord)
            if coord is None and fn.kind != abi.MH_FN_CONSTANT:
                raise ValueError("non-constant TransformAxis without a coordinate")
            ax = Axis(abi.MH_AXIS_ROTATION if name.startswith("rotation")
                      else abi.MH_AXIS_TRANSLATION, tuple(_floats(_text(ta, "axis"))), fn)
            (rot if name.startswith("rotation") else trans).append(ax)
        return rot + trans
    raise NotImplementedError(f"joint type {jtype} not supported")


def _path_points(gp) -> List[PathPoint]:
    pts = []
    ps = gp.find("PathPointSet/objects")
    for p in list(ps):
        body = _text(p, "body") or (_text(p, "socket_parent_frame") or "").split("/")[-1]
        loc = tuple(_floats(_text(p, "location", "0 0 0")))
        if p.tag == "PathPoint":
            pts.append(PathPoint(body, loc, abi.MH_PP_FIXED, name=p.get("name")))
        elif p.tag == "ConditionalPathPoint":
            coord = (_text(p, "coordinate") or _text(p, "socket_coordinate")).split("/")[-1]
            pts.append(PathPoint(body, loc, abi.MH_PP_CONDITIONAL, coord,
                                 tuple(_floats(_text(p, "range"))), name=p.get("name")))
        elif p.tag == "MovingPathPoint":
            fs = {}
            for d in "xyz":
                fel = p.find(f"{d}_location")
                cn = _text(p, f"{d}_coordinate") or _text(p, f"socket_{d}_coordinate")
                cn = cn.split("/")[-1] if cn else None
                fs[d] = parse_function(fel, cn) if fel is not None else None
            pts.append(PathPoint(body, loc, abi.MH_PP_MOVING, fx=fs["x"], fy=fs["y"],
                                 fz=fs["z"], name=p.get("name")))
        else:
            raise NotImplementedError(f"path point {p.tag}")
    return pts


def _path_wraps(gp) -> List[tuple]:
    """GeometryPath PathWrapSet: (wrap object, range begin, range end)."""
    out = []
    ws = gp.find("PathWrapSet/objects") if gp is not None else None
    if ws is None:
        return out
    for w in ws.findall("PathWrap"):
        rng = [int(round(v)) for v in _floats(_text(w, "range", "-1 -1"))] or [-1, -1]
        out.append((_text(w, "wrap_object"), rng[0], rng[1]))
    return out


def _wrap_objects(bel, body: str) -> List[WrapCylinder]:
    """A body's WrapObjectSet (WrapCylinder only)."""
    out = []
    ws = bel.find("WrapObjectSet/objects")
    if ws is None:
        return out
    for w in list(ws):
        if w.tag != "WrapCylinder":
            raise NotImplementedError(f"wrap object {w.tag} ({w.get('name')})")
        out.append(WrapCylinder(
            w.get("name"), body, _float(w, "radius", 0.0), _float(w, "length", 1.0),
            tuple(_floats(_text(w, "xyz_body_rotation", "0 0 0"))),
            tuple(_floats(_text(w, "translation", "0 0 0"))),
            _text(w, "quadrant", "all"), _bool(w, "active", True)))
    return out


def _constraints(mel) -> List[CoordinateCouplerConstraint]:
    """Enabled CoordinateCouplerConstraints with one independent coordinate
    (OpenSim 4: isEnforced; OpenSim 3: isDisabled)."""
    out = []
    cs = mel.find("ConstraintSet/objects")
    if cs is None:
        return out
    for k in list(cs):
        if k.tag != "CoordinateCouplerConstraint":
            raise NotImplementedError(f"constraint {k.tag}")
        if not _bool(k, "isEnforced", True) or _bool(k, "isDisabled", False):
            continue
        ind = (_text(k, "independent_coordinate_names", "") or "").split()
        if len(ind) != 1:
            raise NotImplementedError(f"{k.get('name')}: {len(ind)} independent coordinates")
        fn = parse_function(k.find("coupled_coordinates_function"), ind[0])
        out.append(CoordinateCouplerConstraint(k.get("name"), _text(k, "dependent_coordinate_name"),
                                               fn, _float(k, "scale_factor", 1.0)))
    return out


def _muscle_to_dgf(m, tendon_compliance: Optional[bool],
                   keep_path_wraps: bool = False) -> DeGrooteFregly2016Muscle:
    """DeGrooteFregly2016Muscle::replaceMuscles mapping (.cpp:948-1010).
    replaceMuscles copies the PathPointSet only (.cpp:1007-1020): a replaced
    Millard / Thelen muscle loses its PathWrapSet, as in the reference
    (keep_path_wraps=True keeps it: not the reference's behaviour).  Native
    DeGrooteFregly2016Muscle elements keep theirs."""
    tag = m.tag
    d = DeGrooteFregly2016Muscle(m.get("name"), _path_points(m.find("GeometryPath")))
    if tag == "DeGrooteFregly2016Muscle" or keep_path_wraps:
        d.path_wraps = _path_wraps(m.find("GeometryPath"))
    if tag == "Millard2012EquilibriumMuscle":
        d.default_activation = _float(m, "default_activation", MILLARD_DEFAULTS["default_activation"])
        d.activation_time_constant = _float(m, "activation_time_constant",
                                            MILLARD_DEFAULTS["activation_time_constant"])
        d.deactivation_time_constant = _float(m, "deactivation_time_constant",
                                              MILLARD_DEFAULTS["deactivation_time_constant"])
        d.fiber_damping = _float(m, "fiber_damping", MILLARD_DEFAULTS["fiber_damping"])
        ffl = m.find("FiberForceLengthCurve")
        d.passive_fiber_strain_at_one_norm_force = _float(
            ffl, "strain_at_one_norm_force", MILLARD_DEFAULTS["passive_strain"]) \
            if ffl is not None else MILLARD_DEFAULTS["passive_strain"]
        tfl = m.find("TendonForceLengthCurve")
        d.tendon_strain_at_one_norm_force = _float(
            tfl, "strain_at_one_norm_force", MILLARD_DEFAULTS["tendon_strain"]) \
            if tfl is not None else MILLARD_DEFAULTS["tendon_strain"]
    elif tag == "Thelen2003Muscle":
        d.default_activation = _float(m, "default_activation", 0.05)
        d.activation_time_constant = _float(m, "activation_time_constant", 0.015)
        d.deactivation_time_constant = _float(m, "deactivation_time_constant", 0.05)
        d.fiber_damping = 0.0
        d.passive_fiber_strain_at_one_norm_force = _float(m, "FmaxMuscleStrain", 0.6)
        d.tendon_strain_at_one_norm_force = _float(m, "FmaxTendonStrain", 0.04)
    elif tag == "DeGrooteFregly2016Muscle":
        for k in ("default_activation", "activation_time_constant",
                  "deactivation_time_constant", "fiber_damping",
                  "passive_fiber_strain_at_one_norm_force",
                  "tendon_strain_at_one_norm_force", "active_force_width_scale"):
            v = _float(m, k)
            if v is not None:
                setattr(d, k, v)
        d.ignore_passive_fiber_force = _bool(m, "ignore_passive_fiber_force", False)
        d.tendon_compliance_dynamics_mode = _text(m, "tendon_compliance_dynamics_mode", "explicit")
    else:
        raise NotImplementedError(f"muscle {tag}")
    # Millard2012EquilibriumMuscle keeps its excitation above its
    # minimum_activation (default 0.01): that is the min_control a
    # DeGrooteFregly2016Muscle inherits in replaceMuscles
    # (DeGrooteFregly2016Muscle.cpp:994-995); the MocoInverse golden solution
    # std_testMocoInverse_subject_18musc_solution.sto sits on 0.01.
    lo_default = _float(m, "minimum_activation", 0.01) if tag == "Millard2012EquilibriumMuscle" else 0.0
    d.min_control = _float(m, "min_control", lo_default)
    d.max_control = _float(m, "max_control", 1.0)
    d.max_isometric_force = _float(m, "max_isometric_force", 1000.0)
    d.optimal_fiber_length = _float(m, "optimal_fiber_length", 0.1)
    d.tendon_slack_length = _float(m, "tendon_slack_length", 0.2)
    d.pennation_angle_at_optimal = _float(m, "pennation_angle_at_optimal", 0.0)
    d.max_contraction_velocity = _float(m, "max_contraction_velocity", 10.0)
    d.ignore_tendon_compliance = _bool(m, "ignore_tendon_compliance", False)
    d.ignore_activation_dynamics = _bool(m, "ignore_activation_dynamics", False)
    if tendon_compliance is not None:
        d.ignore_tendon_compliance = not tendon_compliance
    return d


MUSCLE_TAGS = ("Millard2012EquilibriumMuscle", "Thelen2003Muscle",
               "DeGrooteFregly2016Muscle")


def read_osim(path: str, remove_muscles: bool = False,
              tendon_compliance: Optional[bool] = None,
              keep_path_wraps: bool = False) -> Model:
    root = ET.parse(path).getroot()
    mel = root.find("Model")
    model = Model(mel.get("name"), tuple(_floats(_text(mel, "gravity", "0 -9.80665 0"))))
    version = int(root.get("Version", "40000"))
    if version < 40000:
        for b in mel.findall("BodySet/objects/Body"):
            name = b.get("name")
            if name == "ground":
                continue
            inertia = [_float(b, k, 0.0) for k in ("inertia_xx", "inertia_yy", "inertia_zz",
                                                   "inertia_xy", "inertia_xz", "inertia_yz")]
            model.add_body(Body(name, _float(b, "mass", 0.0),
                                tuple(_floats(_text(b, "mass_center", "0 0 0"))), inertia))
            for w in _wrap_objects(b, name):
                model.add_wrap(w)
            jwrap = b.find("Joint")
            jel = list(jwrap)[0] if jwrap is not None and len(list(jwrap)) else None
            if jel is None:
                raise ValueError(f"body {name} has no joint")
            coords = _coordinates(jel)
            model.add_joint(Joint(
                jel.get("name"), _text(jel, "parent_body"), name, coords,
                _axes_for(jel, jel.tag, coords),
                tuple(_floats(_text(jel, "location_in_parent", "0 0 0"))),
                tuple(_floats(_text(jel, "orientation_in_parent", "0 0 0"))),
                tuple(_floats(_text(jel, "location", "0 0 0"))),
                tuple(_floats(_text(jel, "orientation", "0 0 0")))))
    else:
        for b in mel.findall("BodySet/objects/Body"):
            inertia6 = _floats(_text(b, "inertia", "0 0 0 0 0 0"))
            model.add_body(Body(b.get("name"), _float(b, "mass", 0.0),
                                tuple(_floats(_text(b, "mass_center", "0 0 0"))), inertia6))
            for w in _wrap_objects(b, b.get("name")):
                model.add_wrap(w)
        for jel in list(mel.find("JointSet/objects")):
            frames = {f.get("name"): f for f in jel.findall("frames/PhysicalOffsetFrame")}

            def frame_info(sock):
                fname = (_text(jel, sock) or "").split("/")[-1]
                f = frames.get(fname)
                if f is None:
                    return fname, (0, 0, 0), (0, 0, 0)
                parent = (_text(f, "socket_parent") or "").split("/")[-1]
                return (parent, tuple(_floats(_text(f, "translation", "0 0 0"))),
                        tuple(_floats(_text(f, "orientation", "0 0 0"))))
            pname, pl, po = frame_info("socket_parent_frame")
            cname, cl, co = frame_info("socket_child_frame")
            coords = _coordinates(jel)
            model.add_joint(Joint(jel.get("name"), pname, cname, coords,
                                  _axes_for(jel, jel.tag, coords), pl, po, cl, co))
    for k in _constraints(mel):
        model.add_constraint(k)
    # forces, in force-set order
    fs = mel.find("ForceSet/objects")
    if fs is not None:
        for f in list(fs):
            if f.tag in MUSCLE_TAGS:
                if remove_muscles:
                    continue
                if _bool(f, "isDisabled", False) or not _bool(f, "appliesForce", True):
                    continue
                model.add_muscle(_muscle_to_dgf(f, tendon_compliance, keep_path_wraps))
            elif f.tag == "CoordinateActuator":
                model.add_coordinate_actuator(CoordinateActuator(
                    f.get("name"), _text(f, "coordinate"),
                    _float(f, "optimal_force", 1.0),
                    _float(f, "min_control", -math.inf),
                    _float(f, "max_control", math.inf)))
            else:
                raise NotImplementedError(f"force {f.tag} not supported on the hot path")
    return model


def add_reserves(model: Model, optimal_force: float, bound: float = float("nan")):
    """ModelFactory::createReserveActuators (ModelFactory.cpp:265-310): one
    CoordinateActuator per coordinate, in component-list (joint) order."""
    for j in model.joints:
        for c in j.coordinates:
            path = c.path or f"/jointset/{j.name}/{c.name}"
            a = CoordinateActuator("reserve" + path.replace("/", "_"), c.name, optimal_force)
            if not math.isnan(bound):
                a.min_control, a.max_control = -bound, bound
            model.add_coordinate_actuator(a)


def read_storage(path: str):
    """Read an OpenSim .mot/.sto (header ... endheader, then a labelled
    table).  Returns (labels, data[nrow, ncol]) with time in column 0, and
    the header dict."""
    import numpy as np
    header = {}
    with open(path) as fh:
        lines = fh.read().splitlines()
    i = 0
    while i < len(lines) and lines[i].strip().lower() != "endheader":
        if "=" in lines[i]:
            k, v = lines[i].split("=", 1)
            header[k.strip()] = v.strip()
        i += 1
    labels = lines[i + 1].split("\t")
    labels = [l.strip() for l in labels if l.strip() != ""]
    rows = [list(map(float, l.split())) for l in lines[i + 2:] if l.strip()]
    return labels, np.array(rows, float), header
