"""Text description of a MocoStudy at the OpenSim level (model components,
problem goals / bounds / path constraints, solver settings) for the native
C++ problem builder (opensim-moco_amd/csrc/host/mh_builder.{hpp,cpp}), which
lowers it with the same rules as model.py / problem.py.

Whitespace-separated tokens; strings carry no whitespace ("~" = empty /
none); doubles are Python reprs (exact round trip through strtod).  Data
tables travel as the piecewise polynomials the hot path evaluates (the
GCVSpline fit of the samples is done here, by splines.py)."""
from __future__ import annotations

from typing import List

import numpy as np

from .model import CoordinateActuator, DataTable, DeGrooteFregly2016Muscle
from .problem import (Constant, GCVSpline, ImplicitAuxiliaryDerivativesTerm, MocoControlBoundConstraint,
                      MocoControlGoal, MocoFinalTimeGoal, MocoInitialActivationGoal, MocoMarkerFinalGoal,
                      MocoStateTrackingGoal, MocoSumSquaredStateGoal, PiecewiseLinearFunction)
from .splines import gcv_interpolating_ppoly

VERSION = 1


def _s(v) -> str:
    v = "" if v is None else str(v)
    if any(c.isspace() for c in v):
        raise ValueError(f"description strings cannot hold whitespace: {v!r}")
    return v or "~"


def _d(v) -> str:
    return repr(float(v))


def _ds(vals) -> str:
    return " ".join(_d(v) for v in vals)


def _fn(f) -> str:
    if f is None:
        return "F-"
    return " ".join(["F", str(int(f.kind)), _s(f.coord), _d(f.a), _d(f.b), _d(f.scale), str(len(f.x)),
                     _ds(f.x), _ds(f.y)]).replace("  ", " ").strip()


def _table(name: str, cols: List[str], br, cf) -> str:
    br = np.asarray(br, float)
    cf = np.asarray(cf, float)
    return " ".join(["table", _s(name), str(len(cols)), " ".join(_s(c) for c in cols), str(len(br)), _ds(br),
                     str(cf.shape[-1] - 1), _ds(cf.reshape(-1))])


def _fit(t: DataTable, cols=None):
    cols = list(t.columns.keys()) if cols is None else cols
    if t.ppoly is not None:
        return cols, t.ppoly[0], t.ppoly[1]
    br, cf = gcv_interpolating_ppoly(np.asarray(t.times, float),
                                     np.stack([np.asarray(t.columns[c], float) for c in cols], 1), t.degree)
    return cols, br, cf


def _bounds(b) -> str:
    return f"{_d(b.lower)} {_d(b.upper)}"


def _bound_fn(f) -> str:
    if f is None:
        return "none"
    if isinstance(f, Constant):
        return f"const {_d(f.value)}"
    if isinstance(f, PiecewiseLinearFunction):
        return f"pwl {len(f.x)} {_ds(f.x)} {_ds(f.y)}"
    if isinstance(f, GCVSpline):
        br, cf = f.ppoly()
        cf = np.asarray(cf, float)
        return f"spline {len(f.x)} {_ds(f.x)} {len(br)} {_ds(br)} {cf.shape[-1] - 1} {_ds(cf.reshape(-1))}"
    raise TypeError(f"unsupported bound function {type(f).__name__}")


def describe(study) -> str:
    """The description of ``study`` (a MocoStudy)."""
    p, s, m = study.problem, study.solver, study.problem.model
    if s.sparsity_guess is not None or s.sparsity_pattern is not None:
        raise NotImplementedError("sparsity guesses / given patterns do not travel in a description")
    out = [f"mhdesc {VERSION}", f"model {_s(m.name)} {_ds(m.gravity)}"]
    for b in m.bodies.values():
        out.append(f"body {_s(b.name)} {_d(b.mass)} {_ds(b.com)} {_ds(b.inertia)}")
    for j in m.joints:
        out.append(" ".join(["joint", _s(j.name), _s(j.parent), _s(j.child), _ds(j.loc_in_parent),
                             _ds(j.orient_in_parent), _ds(j.loc_in_child), _ds(j.orient_in_child),
                             str(len(j.coordinates)), str(len(j.axes))]))
        for c in j.coordinates:
            out.append(f"coord {_s(c.name)} {_ds(c.range)} {_s(c.motion_type)} {_d(c.default_value)} {_s(c.path)}")
        for a in j.axes:
            out.append(f"axis {int(a.type)} {_ds(a.dir)} {_fn(a.func)}")
    for w in m.wraps.values():
        out.append(" ".join(["wrap", _s(w.name), _s(w.body), _d(w.radius), _d(w.length), _ds(w.xyz_body_rotation),
                             _ds(w.translation), _s(w.quadrant), str(int(bool(w.active)))]))
    for a in m.actuators:
        if isinstance(a, DeGrooteFregly2016Muscle):
            out.append(" ".join(["muscle", _s(a.name), _s(a.path), str(len(a.points)), _ds([
                a.max_isometric_force, a.optimal_fiber_length, a.tendon_slack_length,
                a.pennation_angle_at_optimal, a.max_contraction_velocity, a.activation_time_constant,
                a.deactivation_time_constant, a.default_activation, a.default_normalized_tendon_force,
                a.active_force_width_scale, a.fiber_damping, a.passive_fiber_strain_at_one_norm_force,
                a.tendon_strain_at_one_norm_force]),
                str(int(a.ignore_passive_fiber_force)), str(int(a.ignore_activation_dynamics)),
                str(int(a.ignore_tendon_compliance)), _s(a.tendon_compliance_dynamics_mode),
                _d(a.min_control), _d(a.max_control), str(len(a.path_wraps))]
                + [f"{_s(w)} {int(r0)} {int(r1)}" for (w, r0, r1) in a.path_wraps]))
            for pt in a.points:
                out.append(" ".join(["point", _s(pt.body), _ds(pt.loc), str(int(pt.kind)), _s(pt.coord),
                                     _ds(pt.range), _fn(pt.fx), _fn(pt.fy), _fn(pt.fz), _s(pt.name)]))
        elif isinstance(a, CoordinateActuator):
            out.append(" ".join(["coordact", _s(a.name), _s(a.coordinate), _d(a.optimal_force),
                                 _d(a.min_control), _d(a.max_control), _s(a.path)]))
        else:
            raise TypeError(f"unsupported actuator {type(a).__name__}")
    for f in m.springs:
        out.append(" ".join(["spring", _s(f.name), _s(f.coordinate), _d(f.stiffness), _d(f.rest_length),
                             _d(f.viscosity), _s(f.path)]))
    for mk in m.markers.values():
        out.append(f"marker {_s(mk.name)} {_s(mk.body)} {_ds(mk.location)} {_s(mk.path)}")
    for k in m.constraints:
        out.append(f"constraint {_s(k.name)} {_s(k.dependent)} {_fn(k.function)} {_d(k.scale_factor)}")
    for name, t in m.tables.items():
        cols, br, cf = _fit(t)
        out.append(_table(name, cols, br, cf))
    for e in m.external_forces:
        out.append(" ".join(["extforce", _s(e.name), _s(e.body), _s(e.table), _s(e.force_identifier),
                             _s(e.point_identifier), _s(e.torque_identifier)]))
    # the problem
    out.append(" ".join(["problem", _bounds(p.time_initial), _bounds(p.time_final),
                         _bounds(p.default_speed_bounds), str(int(bool(p.bound_activation_from_excitation))),
                         _bounds(p.kinematic_constraint_bounds), _bounds(p.multiplier_bounds)]))
    for kind, infos in (("stateinfo", p.state_infos), ("controlinfo", p.control_infos)):
        for n, v in infos.items():
            out.append(f"{kind} {_s(n)} {_bounds(v.bounds)} {_bounds(v.initial)} {_bounds(v.final)}")
    for g in p.goals:
        if isinstance(g, MocoControlGoal):
            w = list(g.control_weights.items())
            out.append(" ".join(["goal", "control", _s(g.name), _d(g.weight), str(int(g.exponent)), str(len(w))]
                                + [f"{_s(k)} {_d(v)}" for k, v in w]))
        elif isinstance(g, MocoStateTrackingGoal):
            w = list(g.state_weights.items())
            out.append(" ".join(["goal", "state_tracking", _s(g.name), _d(g.weight), _s(g.reference.name),
                                 str(len(w))] + [f"{_s(k)} {_d(v)}" for k, v in w]))
        elif isinstance(g, MocoFinalTimeGoal):
            out.append(f"goal final_time {_s(g.name)} {_d(g.weight)}")
        elif isinstance(g, MocoSumSquaredStateGoal):
            w = list(g.state_weights.items())
            out.append(" ".join(["goal", "sum_squared_state", _s(g.name), _d(g.weight), str(len(w))]
                                + [f"{_s(k)} {_d(v)}" for k, v in w]))
        elif isinstance(g, MocoInitialActivationGoal):
            out.append(f"goal initial_activation {_s(g.name)} {_s(g.mode)} {_d(g.weight)}")
        elif isinstance(g, MocoMarkerFinalGoal):
            out.append(f"goal marker_final {_s(g.name)} {_d(g.weight)} {_s(g.point_name)} "
                       f"{_ds(g.reference_location)}")
        elif isinstance(g, ImplicitAuxiliaryDerivativesTerm):
            out.append(f"goal aux_derivatives {_s(g.name)} {_d(g.weight)}")
        else:
            raise TypeError(f"unsupported goal {type(g).__name__}")
    for pc in p.path_constraints:
        if not isinstance(pc, MocoControlBoundConstraint):
            raise TypeError(f"unsupported path constraint {type(pc).__name__}")
        out.append(" ".join(["pathcon", _s(pc.name), str(len(pc.control_paths))]
                            + [_s(c) for c in pc.control_paths]
                            + [_bound_fn(pc.lower_bound), _bound_fn(pc.upper_bound),
                               str(int(bool(pc.equality_with_lower)))]))
    for par in p.parameters:
        out.append(" ".join(["parameter", _s(par.name), _s(par.property_name), str(int(par.property_element)),
                             _bounds(par.bounds), str(len(par.component_paths))]
                            + [_s(c) for c in par.component_paths]))
    if p.position_motion is not None:
        kin = p.position_motion
        qpaths = [c.path + "/value" for c in m.coordinates()]
        missing = [q for q in qpaths if q not in kin.columns]
        if missing:
            raise ValueError(f"PositionMotion: no kinematics for {missing}")
        cols, br, cf = _fit(DataTable("__position_motion", np.asarray(kin.times, float),
                                      {q: np.asarray(kin.columns[q], float) for q in qpaths},
                                      degree=kin.degree))
        out.append("position_motion " + _table("__position_motion", cols, br, cf))
    out.append(" ".join([
        "solver", str(int(s.num_mesh_intervals)), _s(s.transcription_scheme),
        str(int(bool(s.interpolate_control_midpoints))), _s(s.optim_finite_difference_scheme), _d(s.fd_step),
        str(int(s.device)), _s(s.multibody_dynamics_mode), _ds(s.implicit_multibody_acceleration_bounds),
        _ds(s.implicit_auxiliary_derivative_bounds), str(int(bool(s.enforce_constraint_derivatives))),
        str(int(bool(s.minimize_lagrange_multipliers))), _d(s.lagrange_multiplier_weight), _s(s.jacobian_mode),
        _ds(s.velocity_correction_bounds), _s(s.optim_sparsity_detection),
        str(int(s.optim_sparsity_detection_random_count)), _s(s.optim_sparsity_detection_rule)]))
    out.append("end")
    return "\n".join(out) + "\n"


def write_description(study, path: str) -> None:
    with open(path, "w") as fh:
        fh.write(describe(study))

