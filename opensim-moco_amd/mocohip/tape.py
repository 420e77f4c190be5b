"""Problem tape files: a compiled MocoProblemRep (the mh_problem the C ABI
receives) plus the solver options, written to one binary file so that
native host code (opensim-moco_amd/csrc/host/mh_driver.cpp, or a C++
MocoSolver plugin) can drive libmocohip without Python.

Layout (little endian, x86-64 struct layout of include/mocohip.h):
  magic "MHTAPE01", int32 version, int32 NS, int32 NC, mh_options,
  the 12 mh_model counts, gravity[3], time bounds (2 x mh_bounds),
  ngoals, nterms, then the arrays in mh_model / mh_problem field order,
  each as (int64 byte count, bytes); version 2 appends npath and the
  mh_path_equation array, then the sparsity-detection guess (n doubles or
  empty), the given callback sparsity (bytes or empty) and the prescribed
  kinematics (table index, per-coordinate columns); version 3 appends the
  endpoint-constraint equations (mh_problem.nendpoint/endpoint); version 4
  (ABI v4: mh_options grew) appends the kinematic constraints
  (mh_model.nconstraints/constraints) and the multiplier and
  kinematic-constraint bounds; version 5 (ABI v5) appends the wrap surfaces
  and PathWraps (mh_model.nwraps/wraps, npathwraps/pathwraps); version 6
  carries ABI v6's mh_options (+ sparsity_rule); version 7 ABI v7's (the
  rule's values swapped: the reference's any-change rule is 0); version 8
  ABI v8's (coloring_order) and appends the springs (mh_model.nsprings /
  springs) and the MocoParameters (nparameters + bounds, nparameter_targets
  + targets); from version 8 the initial-guess blob is the whole iterate (n
  doubles, what mh_create reads; mh_driver checks it against
  mh_get_nlp_info_for).  Readers accept versions 4 to 8 (a version-6 tape's
  rule is mapped to v7's value)."""
from __future__ import annotations

import ctypes as C
import struct

from . import abi

MAGIC = b"MHTAPE01"
VERSION = 8   # 2: + path constraints; 3: + endpoint constraints; 4: + kinematic constraints; 5: + wraps;
#               6: ABI v6 mh_options; 7: ABI v7 (sparsity_rule values swapped); 8: ABI v8 (springs,
#               parameters, the guess blob = n doubles)

# (field, element type, count attribute of mh_model / None for problem arrays)
_MODEL_ARRAYS = [
    ("bodies", abi.mh_body, "nbodies"), ("axes", abi.mh_axis, "naxes"),
    ("functions", abi.mh_function, "nfunctions"), ("knot_x", C.c_double, "nknots"),
    ("knot_y", C.c_double, "nknots"), ("muscles", abi.mh_muscle, "nmuscles"),
    ("points", abi.mh_path_point, "npoints"), ("actuators", abi.mh_actuator, "nactuators"),
    ("tables", abi.mh_table, "ntables"), ("table_breaks", C.c_double, "nbreaks"),
    ("table_coefs", C.c_double, "ncoefs"), ("external", abi.mh_external_force, "nexternal"),
]
_COUNTS = ["nq", "nbodies", "naxes", "nfunctions", "nknots", "nmuscles", "npoints",
           "nactuators", "ntables", "nbreaks", "ncoefs", "nexternal"]


def _blob(ptr, ctype, count: int) -> bytes:
    if count <= 0 or not ptr:
        return b""
    return C.string_at(ptr, C.sizeof(ctype) * count)


def write_tape(rep, opts: abi.mh_options, path: str) -> None:
    """Serialize ``rep`` (a ProblemRep) and ``opts`` to ``path``."""
    p = rep.struct
    m = p.model
    ns, nc = len(rep.state_names), len(rep.control_names)
    # pointers inside mh_options do not travel: the sparsity guess is a blob
    guess = b""
    implicit = opts.multibody_dynamics_mode == abi.MH_DYNAMICS_IMPLICIT
    presc = bool(p.prescribed_kinematics)
    nar = getattr(rep, "num_aux_residuals", 0)
    ndv = (m.nq if implicit and not presc else 0) + nar
    if opts.sparsity_guess:
        # the whole iterate: n doubles (mh_options.sparsity_guess)
        info = abi.mh_nlp_info()
        lib = abi.load_mocohip()
        if lib.mh_get_nlp_info_for(C.byref(p), C.byref(opts), C.byref(info)) != 0:
            raise RuntimeError(lib.mh_last_error().decode())
        size = getattr(opts, "_guess_size", None)
        if size is not None and size != int(info.n):
            raise ValueError(f"sparsity_guess has {size} values, the problem has n = {int(info.n)}")
        guess = C.string_at(opts.sparsity_guess, 8 * int(info.n))
    pattern = b""
    if opts.sparsity_pattern:
        # mh_get_callback_sparsity layout: NO DAE outputs and the path
        # equations (W flags each), the endpoint equations (2 W flags each)
        W = 1 + ns + nc + ndv + (m.nconstraints if presc else 0)   # + multipliers
        nz = ns if presc else ns - 2 * m.nq
        no = m.nq + nz + nar
        pattern = C.string_at(opts.sparsity_pattern, (no + p.npath + 2 * p.nendpoint) * W)
    o2 = abi.mh_options.from_buffer_copy(bytes(opts))
    o2.sparsity_guess = None
    o2.sparsity_pattern = None
    out = [MAGIC, struct.pack("<iii", VERSION, ns, nc), bytes(o2)]
    out.append(struct.pack("<12i", *[getattr(m, k) for k in _COUNTS]))
    out.append(struct.pack("<3d", *m.gravity))
    out.append(bytes(p.time_initial) + bytes(p.time_final))
    out.append(struct.pack("<ii", p.ngoals, p.nterms))
    blobs = [_blob(getattr(m, f), t, getattr(m, cnt)) for f, t, cnt in _MODEL_ARRAYS]
    blobs += [_blob(p.state_infos, abi.mh_variable_info, ns),
              _blob(p.control_infos, abi.mh_variable_info, nc),
              _blob(p.goals, abi.mh_goal, p.ngoals),
              _blob(p.goal_index, C.c_int32, p.nterms),
              _blob(p.goal_column, C.c_int32, p.nterms),
              _blob(p.goal_weight, C.c_double, p.nterms)]
    for b in blobs:
        out.append(struct.pack("<q", len(b)))
        out.append(b)
    pb = _blob(p.path, abi.mh_path_equation, p.npath)
    out += [struct.pack("<i", p.npath), struct.pack("<q", len(pb)), pb]
    out += [struct.pack("<q", len(guess)), guess, struct.pack("<q", len(pattern)), pattern]
    kc = _blob(p.kinematics_column, C.c_int32, m.nq) if p.prescribed_kinematics else b""
    out += [struct.pack("<ii", p.prescribed_kinematics, p.kinematics_table), struct.pack("<q", len(kc)), kc]
    eb = _blob(p.endpoint, abi.mh_endpoint_equation, p.nendpoint)
    out += [struct.pack("<i", p.nendpoint), struct.pack("<q", len(eb)), eb]
    kb = _blob(m.constraints, abi.mh_constraint, m.nconstraints)
    out += [struct.pack("<i", m.nconstraints), struct.pack("<q", len(kb)), kb,
            bytes(p.multiplier_bounds), bytes(p.kinematic_constraint_bounds)]
    wb = _blob(m.wraps, abi.mh_wrap_object, m.nwraps)
    pw = _blob(m.pathwraps, abi.mh_path_wrap, m.npathwraps)
    out += [struct.pack("<i", m.nwraps), struct.pack("<q", len(wb)), wb,
            struct.pack("<i", m.npathwraps), struct.pack("<q", len(pw)), pw]
    sb = _blob(m.springs, abi.mh_spring, m.nsprings)
    pbnd = _blob(p.parameter_bounds, abi.mh_bounds, p.nparameters)
    ptg = _blob(p.parameter_targets, abi.mh_parameter_target, p.nparameter_targets)
    out += [struct.pack("<i", m.nsprings), struct.pack("<q", len(sb)), sb,
            struct.pack("<i", p.nparameters), struct.pack("<q", len(pbnd)), pbnd,
            struct.pack("<i", p.nparameter_targets), struct.pack("<q", len(ptg)), ptg]
    with open(path, "wb") as fh:
        fh.write(b"".join(out))
