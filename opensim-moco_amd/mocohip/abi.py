"""ctypes mirror of include/mocohip.h (the C-ABI drop-in boundary).

The structs here are byte-for-byte the ones declared in include/mocohip.h;
``tests/test_abi.py`` checks sizes and field offsets against the header.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                     # opensim-moco_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)

MH_OK, MH_ERR_INVALID, MH_ERR_HIP, MH_ERR_UNSUPPORTED, MH_ERR_ALLOC = range(5)

MH_FN_CONSTANT, MH_FN_LINEAR, MH_FN_SIMMSPLINE = 0, 1, 2
MH_AXIS_ROTATION, MH_AXIS_TRANSLATION = 0, 1
MH_PP_FIXED, MH_PP_CONDITIONAL, MH_PP_MOVING = 0, 1, 2
MH_ACT_MUSCLE, MH_ACT_COORDINATE = 0, 1
MH_GOAL_CONTROL, MH_GOAL_STATE_TRACKING, MH_GOAL_FINAL_TIME, \
    MH_GOAL_SUM_SQUARED_STATE, MH_GOAL_AUX_DERIVATIVES, MH_GOAL_MARKER_FINAL = 0, 1, 2, 3, 4, 5
MH_HERMITE_SIMPSON, MH_TRAPEZOIDAL = 0, 1
MH_DYNAMICS_EXPLICIT, MH_DYNAMICS_IMPLICIT = 0, 1
MH_FD_CENTRAL, MH_FD_FORWARD, MH_FD_BACKWARD = 0, 1, 2

i32 = C.c_int32
f64 = C.c_double
P = C.POINTER


class mh_function(C.Structure):
    _fields_ = [("kind", i32), ("coord", i32), ("knot_begin", i32),
                ("knot_count", i32), ("a", f64), ("b", f64), ("scale", f64),
                ("reserved", f64)]


class mh_axis(C.Structure):
    _fields_ = [("type", i32), ("func", i32), ("dir", f64 * 3)]


class mh_body(C.Structure):
    _fields_ = [("parent", i32), ("axis_begin", i32), ("axis_count", i32),
                ("reserved", i32), ("mass", f64), ("com", f64 * 3),
                ("inertia", f64 * 6), ("R_PF", f64 * 9), ("p_PF", f64 * 3),
                ("R_BM", f64 * 9), ("p_BM", f64 * 3)]


class mh_path_point(C.Structure):
    _fields_ = [("kind", i32), ("body", i32), ("coord", i32), ("fx", i32),
                ("fy", i32), ("fz", i32), ("loc", f64 * 3),
                ("range", f64 * 2)]


class mh_muscle(C.Structure):
    _fields_ = [("point_begin", i32), ("point_count", i32),
                ("ignore_activation_dynamics", i32),
                ("ignore_tendon_compliance", i32),
                ("ignore_passive_fiber_force", i32),
                ("tendon_dynamics_implicit", i32),
                ("max_isometric_force", f64), ("optimal_fiber_length", f64),
                ("tendon_slack_length", f64),
                ("pennation_angle_at_optimal", f64),
                ("max_contraction_velocity", f64),
                ("activation_time_constant", f64),
                ("deactivation_time_constant", f64), ("fiber_damping", f64),
                ("passive_fiber_strain_at_one_norm_force", f64),
                ("tendon_strain_at_one_norm_force", f64),
                ("active_force_width_scale", f64)]


class mh_actuator(C.Structure):
    _fields_ = [("kind", i32), ("target", i32), ("optimal_force", f64)]


class mh_table(C.Structure):
    _fields_ = [("nseg", i32), ("degree", i32), ("ncol", i32),
                ("break_begin", i32), ("coef_begin", i32), ("reserved", i32)]


class mh_external_force(C.Structure):
    _fields_ = [("body", i32), ("table", i32), ("force_col", i32),
                ("point_col", i32), ("torque_col", i32), ("reserved", i32)]


MH_KC_COORDINATE_COUPLER = 0
MH_JACOBIAN_CALLBACK_FD, MH_JACOBIAN_GLOBAL_SEEDS = 0, 1
MH_COLORING_SMALLEST_LAST, MH_COLORING_NATURAL = 0, 1


class mh_constraint(C.Structure):
    _fields_ = [("kind", i32), ("dependent", i32), ("func", i32), ("reserved", i32),
                ("scale", f64)]


MH_WRAP_CYLINDER = 0


class mh_wrap_object(C.Structure):
    _fields_ = [("kind", i32), ("body", i32), ("wrap_axis", i32), ("wrap_sign", i32),
                ("R_BW", f64 * 9), ("p_BW", f64 * 3), ("radius", f64), ("length", f64)]


class mh_path_wrap(C.Structure):
    _fields_ = [("muscle", i32), ("wrap", i32), ("range_begin", i32), ("range_end", i32)]


class mh_spring(C.Structure):
    _fields_ = [("coord", i32), ("reserved", i32), ("stiffness", f64), ("rest_length", f64),
                ("viscosity", f64)]


MH_PARAM_BODY_MASS, MH_PARAM_BODY_MASS_CENTER, MH_PARAM_BODY_INERTIA, MH_PARAM_SPRING_STIFFNESS, \
    MH_PARAM_SPRING_REST_LENGTH, MH_PARAM_SPRING_VISCOSITY, MH_PARAM_ACTUATOR_OPTIMAL_FORCE, \
    MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE = range(8)


class mh_parameter_target(C.Structure):
    _fields_ = [("parameter", i32), ("kind", i32), ("index", i32), ("element", i32)]


class mh_model(C.Structure):
    _fields_ = [("nq", i32), ("nbodies", i32), ("naxes", i32),
                ("nfunctions", i32), ("nknots", i32), ("nmuscles", i32),
                ("npoints", i32), ("nactuators", i32), ("ntables", i32),
                ("nbreaks", i32), ("ncoefs", i32), ("nexternal", i32),
                ("gravity", f64 * 3),
                ("bodies", P(mh_body)), ("axes", P(mh_axis)),
                ("functions", P(mh_function)), ("knot_x", P(f64)),
                ("knot_y", P(f64)), ("muscles", P(mh_muscle)),
                ("points", P(mh_path_point)), ("actuators", P(mh_actuator)),
                ("tables", P(mh_table)), ("table_breaks", P(f64)),
                ("table_coefs", P(f64)),
                ("external", P(mh_external_force)),
                ("nconstraints", i32), ("reserved_kc", i32), ("constraints", P(mh_constraint)),
                ("nwraps", i32), ("npathwraps", i32), ("wraps", P(mh_wrap_object)),
                ("pathwraps", P(mh_path_wrap)),
                ("nsprings", i32), ("reserved_sp", i32), ("springs", P(mh_spring))]


class mh_bounds(C.Structure):
    _fields_ = [("lower", f64), ("upper", f64)]


class mh_variable_info(C.Structure):
    _fields_ = [("bounds", mh_bounds), ("initial", mh_bounds),
                ("final", mh_bounds)]


class mh_goal(C.Structure):
    _fields_ = [("kind", i32), ("table", i32), ("term_begin", i32),
                ("term_count", i32), ("exponent", i32), ("reserved", i32),
                ("weight", f64)]


MH_ABI_VERSION = 8     # include/mocohip.h
MH_PATH_CONTROL_BOUND = 0
MH_ENDPOINT_INITIAL_ACTIVATION = 0


class mh_endpoint_equation(C.Structure):
    _fields_ = [("kind", i32), ("index_a", i32), ("index_b", i32), ("reserved", i32),
                ("g", mh_bounds)]


class mh_path_equation(C.Structure):
    _fields_ = [("kind", i32), ("index", i32), ("table", i32), ("column", i32),
                ("value", f64), ("g", mh_bounds)]


class mh_problem(C.Structure):
    _fields_ = [("model", mh_model), ("time_initial", mh_bounds),
                ("time_final", mh_bounds),
                ("state_infos", P(mh_variable_info)),
                ("control_infos", P(mh_variable_info)),
                ("ngoals", i32), ("nterms", i32), ("goals", P(mh_goal)),
                ("goal_index", P(i32)), ("goal_column", P(i32)),
                ("goal_weight", P(f64)),
                ("npath", i32), ("reserved", i32), ("path", P(mh_path_equation)),
                ("prescribed_kinematics", i32), ("kinematics_table", i32),
                ("kinematics_column", P(i32)),
                ("nendpoint", i32), ("reserved2", i32), ("endpoint", P(mh_endpoint_equation)),
                ("multiplier_bounds", mh_bounds), ("kinematic_constraint_bounds", mh_bounds),
                ("nparameters", i32), ("nparameter_targets", i32),
                ("parameter_bounds", P(mh_bounds)), ("parameter_targets", P(mh_parameter_target))]


class mh_options(C.Structure):
    _fields_ = [("num_mesh_intervals", i32), ("transcription", i32),
                ("interpolate_control_midpoints", i32),
                ("finite_difference_scheme", i32), ("fd_step", f64),
                ("interval_begin", i32), ("interval_end", i32),
                ("device", i32), ("multibody_dynamics_mode", i32),
                ("implicit_accel_bounds", f64 * 2),
                ("sparsity_detection", i32), ("sparsity_random_count", i32),
                ("sparsity_guess", P(f64)), ("sparsity_pattern", P(C.c_uint8)),
                ("implicit_aux_bounds", f64 * 2),
                ("ignore_constraint_derivatives", i32), ("minimize_lagrange_multipliers", i32),
                ("velocity_correction_bounds", f64 * 2), ("lagrange_multiplier_weight", f64),
                ("jacobian_mode", i32), ("coloring_order", i32),
                ("sparsity_rule", i32), ("reserved_sr", i32)]


MH_SPARSITY_NONE, MH_SPARSITY_RANDOM, MH_SPARSITY_INITIAL_GUESS, MH_SPARSITY_GIVEN = 0, 1, 2, 3
MH_SPARSITY_RULE_ANY_CHANGE, MH_SPARSITY_RULE_ROBUST = 0, 1   # ABI v7: the reference's rule is 0
MH_SPARSITY_ROBUST_TOL = 1e-12


class mh_nlp_info(C.Structure):
    _fields_ = [("n", C.c_int64), ("m", C.c_int64), ("nnz_jac_g", C.c_int64),
                ("nnz_h_lag", C.c_int64), ("num_grid_points", C.c_int64),
                ("num_states", C.c_int64), ("num_controls", C.c_int64),
                ("row_begin", C.c_int64), ("row_end", C.c_int64),
                ("nnz_begin", C.c_int64), ("nnz_end", C.c_int64)]


# Exported entry points of libmocohip.so and their signatures; the
# C-ABI test checks every one is exported (and matches include/mocohip.h).
MOCOHIP_SYMBOLS = {
    "mh_abi_version": (i32, []),
    "mh_eval_objective_terms": (i32, [C.c_void_p, P(f64), P(f64), P(i32)]),
    "mh_build_id": (C.c_char_p, []),
    "mh_backend_for": (i32, [P(mh_problem), P(mh_options), C.c_char_p, i32]),
    "mh_last_error": (C.c_char_p, []),
    "mh_create": (i32, [P(mh_problem), P(mh_options), P(C.c_void_p)]),
    "mh_get_nlp_info_for": (i32, [P(mh_problem), P(mh_options), P(mh_nlp_info)]),
    "mh_destroy": (None, [C.c_void_p]),
    "mh_get_nlp_info": (i32, [C.c_void_p, P(mh_nlp_info)]),
    "mh_get_bounds": (i32, [C.c_void_p, P(f64), P(f64), P(f64), P(f64)]),
    "mh_get_initial_guess_from_bounds": (i32, [C.c_void_p, P(f64)]),
    "mh_get_random_iterate": (i32, [C.c_void_p, P(f64), P(f64)]),
    "mh_get_jac_structure": (i32, [C.c_void_p, P(i32), P(i32)]),
    "mh_eval_f": (i32, [C.c_void_p, P(f64), C.c_int, P(f64)]),
    "mh_eval_grad_f": (i32, [C.c_void_p, P(f64), C.c_int, P(f64)]),
    "mh_eval_f_partial": (i32, [C.c_void_p, P(f64), P(f64)]),
    "mh_eval_grad_f_partial": (i32, [C.c_void_p, P(f64), P(f64)]),
    "mh_eval_g": (i32, [C.c_void_p, P(f64), C.c_int, P(f64)]),
    "mh_eval_jac_g": (i32, [C.c_void_p, P(f64), C.c_int, P(f64)]),
    "mh_eval_g_device": (i32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mh_eval_jac_g_device": (i32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mh_eval_g_jac_g": (i32, [C.c_void_p, P(f64), P(f64), P(f64)]),
    "mh_eval_g_jac_g_device": (i32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mh_tnlp_eval_g_device": (i32, [C.c_void_p, C.c_void_p, i32, C.c_void_p]),
    "mh_tnlp_eval_jac_g_device": (i32, [C.c_void_p, C.c_void_p, i32, C.c_void_p]),
    "mh_eval_dae": (i32, [C.c_void_p, i32, P(f64), P(f64)]),
    "mh_set_timing": (i32, [C.c_void_p, i32]),
    "mh_get_backend_flags": (i32, [C.c_void_p, C.c_char_p, i32]),
    "mh_last_timings": (i32, [C.c_void_p, P(f64)]),
    "mh_get_backend": (i32, [C.c_void_p, C.c_char_p, i32, P(f64), P(C.c_uint64)]),
    "mh_model_hash": (i32, [P(mh_model), P(C.c_uint64)]),
    "mh_get_callback_sparsity": (i32, [C.c_void_p, P(C.c_uint8), C.c_int64]),
    "mh_get_work": (i32, [C.c_void_p, P(f64)]),
    "mh_color_jacobian": (i32, [C.c_int64, C.c_int64, C.c_int64, P(i32), P(i32), P(i32), P(i32)]),
    "mh_color_jacobian_ordered": (i32, [C.c_int64, C.c_int64, C.c_int64, P(i32), P(i32), i32, P(i32),
                                        P(i32)]),
    "mh_get_jacobian_seeds": (i32, [C.c_void_p, P(i32), P(i32)]),
    "mh_debug_jacobian_lanes": (i32, [C.c_void_p, P(f64), P(f64), P(f64)]),
    "mh_debug_time_stages": (i32, [C.c_void_p, C.c_void_p, i32, i32, P(f64)]),
    "mh_set_stream": (i32, [C.c_void_p, C.c_void_p]),
    "mh_set_async": (i32, [C.c_void_p, i32]),
    "mh_batch_create": (i32, [C.POINTER(C.c_void_p), i32, C.POINTER(C.c_void_p)]),
    "mh_batch_destroy": (None, [C.c_void_p]),
    "mh_batch_eval_g_device": (i32, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "mh_batch_eval_jac_g_device": (i32, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "mh_batch_eval_g_jac_g_device": (i32, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_void_p)]),
    "mh_batch_set_group_results_global": (i32, [C.c_void_p, i32]),
    "mh_synchronize": (i32, [C.c_void_p]),
}

ORACLE_SYMBOLS = {
    "orc_last_error": (C.c_char_p, []),
    "orc_create": (i32, [P(mh_problem), P(mh_options), P(C.c_void_p)]),
    "orc_destroy": (None, [C.c_void_p]),
    "orc_set_threads": (None, [C.c_void_p, C.c_int]),
    "orc_get_nlp_info": (i32, [C.c_void_p, P(mh_nlp_info)]),
    "orc_get_bounds": (i32, [C.c_void_p, P(f64), P(f64), P(f64), P(f64)]),
    "orc_get_initial_guess_from_bounds": (i32, [C.c_void_p, P(f64)]),
    "orc_get_random_iterate": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_get_jac_structure": (i32, [C.c_void_p, P(i32), P(i32)]),
    "orc_eval_f": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_grad_f": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_f_partial": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_grad_f_partial": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_g": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_jac_g": (i32, [C.c_void_p, P(f64), P(f64)]),
    "orc_eval_dae": (i32, [C.c_void_p, i32, P(f64), P(f64)]),
    "orc_eval_dae_params": (i32, [C.c_void_p, P(f64), i32, f64, i32, P(f64), P(f64)]),
    "orc_dgf_curve": (f64, [P(mh_muscle), C.c_int, f64]),
    "orc_muscle_length_speed": (i32, [C.c_void_p, C.c_int, P(f64), P(f64),
                                      P(f64)]),
    "orc_muscle_path": (i32, [C.c_void_p, C.c_int, P(f64), P(f64), C.c_int, P(C.c_int), P(f64)]),
    "orc_eval_function": (i32, [C.c_void_p, C.c_int, f64, P(f64)]),
    "orc_get_callback_sparsity": (i32, [C.c_void_p, P(C.c_uint8), C.c_int64]),
    "orc_get_jacobian_seeds": (i32, [C.c_void_p, P(i32), P(i32)]),
    "orc_color_jacobian": (i32, [C.c_int64, C.c_int64, C.c_int64, P(i32), P(i32), i32, P(i32), P(i32)]),
    "orc_assemble_from_lanes": (i32, [C.c_void_p, P(f64), P(f64), P(f64), P(f64), P(f64)]),
}

LIBMOCOHIP_PATH = os.path.join(PKG_ROOT, "csrc", "build", "libmocohip.so")
LIBORACLE_PATH = os.path.join(REPO_ROOT, "oracle", "build", "liboracle.so")


def _bind(lib, table):
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_libs: dict = {}


# include/mocohip_kkt.h: the device KKT module (mocohip/kkt.py)
MOCOHIP_KKT_SYMBOLS = {
    "mh_kkt_create": (i32, [C.c_void_p, C.c_void_p, P(C.c_void_p)]),
    "mh_kkt_destroy": (None, [C.c_void_p]),
    "mh_kkt_set_row_scale": (i32, [C.c_void_p, P(f64)]),
    "mh_kkt_eval_jacobian": (i32, [C.c_void_p, P(f64)]),
    "mh_kkt_get_values": (i32, [C.c_void_p, P(f64)]),
    "mh_kkt_get_dense": (i32, [C.c_void_p, P(f64)]),
    "mh_kkt_factor": (i32, [C.c_void_p, P(f64), P(f64), P(i32)]),
    "mh_kkt_solve": (i32, [C.c_void_p, i32, P(f64), P(f64)]),
    "mh_kkt_jmul": (i32, [C.c_void_p, i32, P(f64), P(f64)]),
    "mh_kkt_jtmul": (i32, [C.c_void_p, i32, P(f64), P(f64)]),
    "mh_kkt_assemble": (i32, [C.c_void_p]),
    "mh_kkt_bind_values": (i32, [C.c_void_p, C.c_void_p]),
    "mh_kkt_shard_range": (i32, [C.c_void_p, P(C.c_int64), P(C.c_int64)]),
}


def load_mocohip(path: str | None = None):
    """Load the product library.  Raises if it is missing: there is no CPU
    fallback for the hot path."""
    path = path or LIBMOCOHIP_PATH
    if path not in _libs:
        # One HIP runtime per process: if PyTorch is installed, load it first so
        # libmocohip binds (by soname) to the same libamdhip64 as torch and
        # torch-allocated device pointers can be passed to the *_device calls.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(path):
            raise RuntimeError(
                f"libmocohip.so not built at {path}; run "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        lib = _bind(C.CDLL(path), {**MOCOHIP_SYMBOLS, **MOCOHIP_KKT_SYMBOLS})
        if lib.mh_abi_version() != MH_ABI_VERSION:
            raise RuntimeError(f"{path}: ABI version {lib.mh_abi_version()}, "
                               f"this binding expects {MH_ABI_VERSION}; rebuild")
        want = tree_build_id()
        have = lib.mh_build_id().decode()
        if want is not None and have != want:
            raise RuntimeError(f"{path} was built from other sources (build id {have}, the tree's "
                               f"is {want}); rebuild with __graft_entry__.build()")
        _libs[path] = lib
    return _libs[path]


def tree_build_id():
    """The source hash of the tree (tools/build_id.py), or None when the
    sources are not present."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    tool = os.path.join(root, "tools", "build_id.py")
    if not os.path.exists(tool):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mh_build_id", tool)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.build_id()


def load_oracle(path: str | None = None):
    """Load the CPU oracle (test infrastructure only)."""
    path = path or LIBORACLE_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"liboracle.so not built at {path}")
        _libs[path] = _bind(C.CDLL(path), ORACLE_SYMBOLS)
    return _libs[path]


def _fnv1a(h: int, data: bytes) -> int:
    for b in data:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def model_hash(m: "mh_model") -> int:
    """mh_model_hash (mocohip.hip model_hash) restated on the host: FNV-1a
    64 over the model tape's counts, gravity, bodies, axes, functions, knots,
    muscles, path points, actuators, external loads and their tables' shapes
    (the keys of the generated back ends; tests/test_abi.py checks it against
    the library)."""
    h = 1469598103934665603
    h = _fnv1a(h, bytes((i32 * 9)(m.nq, m.nbodies, m.naxes, m.nfunctions, m.nknots,
                                    m.nmuscles, m.npoints, m.nactuators, m.nexternal)))
    h = _fnv1a(h, bytes(m.gravity))

    def arr(ptr, T, n):
        return C.string_at(ptr, C.sizeof(T) * n) if n > 0 else b""
    for ptr, T, n in ((m.bodies, mh_body, m.nbodies), (m.axes, mh_axis, m.naxes),
                      (m.functions, mh_function, m.nfunctions), (m.knot_x, f64, m.nknots),
                      (m.knot_y, f64, m.nknots), (m.muscles, mh_muscle, m.nmuscles),
                      (m.points, mh_path_point, m.npoints),
                      (m.actuators, mh_actuator, m.nactuators),
                      (m.external, mh_external_force, m.nexternal)):
        h = _fnv1a(h, arr(ptr, T, n))
    for e in range(m.nexternal):
        t = m.external[e].table
        if 0 <= t < m.ntables:
            h = _fnv1a(h, bytes((i32 * 2)(m.tables[t].degree, m.tables[t].ncol)))
    if m.nwraps > 0 or m.npathwraps > 0:
        h = _fnv1a(h, bytes((i32 * 2)(m.nwraps, m.npathwraps)))
        h = _fnv1a(h, arr(m.wraps, mh_wrap_object, m.nwraps))
        h = _fnv1a(h, arr(m.pathwraps, mh_path_wrap, m.npathwraps))
    return h


def dptr(a):
    """ctypes double* of a contiguous float64 numpy array."""
    return a.ctypes.data_as(P(f64))


def iptr(a):
    return a.ctypes.data_as(P(i32))
