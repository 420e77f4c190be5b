/* mocohip.h — C ABI of the MI355X-native Moco direct-collocation hot path.
 *
 * This is the drop-in boundary.  A host NLP solver
 * (IPOPT's TNLP, or the Python MocoHipSolver mirror) drives it exactly the
 * way tropter's IPOPTSolver::TNLP drives its problem:
 *
 *   reference callback                      replaced by
 *   ------------------------------------    ---------------------------------
 *   TNLP::get_nlp_info                      mh_get_nlp_info
 *     (tropter/tropter/optimization/IPOPTSolver.cpp:302-335)
 *   TNLP::get_bounds_info                   mh_get_bounds
 *     (IPOPTSolver.cpp:337-383; bounds rules CasOCTranscription.cpp:173-250)
 *   TNLP::get_starting_point                mh_get_initial_guess_from_bounds,
 *                                           mh_get_random_iterate
 *     (IPOPTSolver.cpp:385-399; CasOCTranscription.cpp:1123-1177)
 *   TNLP::eval_f / eval_grad_f              mh_eval_f / mh_eval_grad_f
 *     (IPOPTSolver.cpp:401-416)
 *   TNLP::eval_g                            mh_eval_g
 *     (IPOPTSolver.cpp:417-427; CasOCTranscription.cpp:253-446)
 *   TNLP::eval_jac_g (values==nullptr)      mh_get_jac_structure
 *   TNLP::eval_jac_g (values!=nullptr)      mh_eval_jac_g
 *     (IPOPTSolver.cpp:428-447; ProblemDecorator_double.cpp:261-291)
 *
 * The per-grid-point callbacks of CasOC::Problem
 * (Moco/Moco/MocoCasADiSolver/CasOCProblem.h:313-332) are not exported
 * individually: they are the device kernels behind these entry points.
 *
 * Conventions
 *  - All arithmetic is IEEE binary64.
 *  - Indices are 0-based (IPOPT C_STYLE).
 *  - Host-pointer entry points copy x to the device and results back; the
 *    *_device variants take device pointers (e.g. torch tensor data_ptr())
 *    and never touch host memory.  All work is ordered on one HIP stream:
 *    the context's own, or the caller's (mh_set_stream).  By default every
 *    entry returns after its results are complete; with mh_set_async(ctx,
 *    1) the *_device entries return once their kernels are enqueued, and
 *    the caller orders consumers on that stream or calls mh_synchronize.
 *  - Every function returns MH_OK (0) or an error code; mh_last_error()
 *    gives a thread-local message.  A context is used by one host thread at
 *    a time; distinct contexts may run concurrently (one HIP stream each).
 *  - There is NO CPU fallback: mh_create fails with MH_ERR_HIP when no
 *    gfx950 device is usable.
 */
#ifndef MOCOHIP_H
#define MOCOHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_ABI_VERSION 8

enum mh_status {
    MH_OK = 0,
    MH_ERR_INVALID = 1,     /* bad argument / malformed problem            */
    MH_ERR_HIP = 2,         /* HIP runtime failure or no usable device      */
    MH_ERR_UNSUPPORTED = 3, /* feature outside the implemented hot path     */
    MH_ERR_ALLOC = 4
};

/* ------------------------------------------------------------------------ */
/* Model description ("model tape").  Plain structs of int32/double so that  */
/* ctypes, cgo or JNI can fill them.  Produced by the host-side model        */
/* compiler (opensim-moco_amd/mocohip/model.py) from an OpenSim model.       */
/* ------------------------------------------------------------------------ */

/* Scalar function of (at most) one generalized coordinate: the subset of
 * OpenSim::Function used by CustomJoint TransformAxis and MovingPathPoint
 * (Constant, LinearFunction, SimmSpline, MultiplierFunction(SimmSpline)). */
enum mh_function_kind {
    MH_FN_CONSTANT = 0,   /* value = a                                   */
    MH_FN_LINEAR = 1,     /* value = scale * (a * q + b)                  */
    MH_FN_SIMMSPLINE = 2  /* value = scale * SimmSpline(knots)(q)         */
};
typedef struct mh_function {
    int32_t kind;
    int32_t coord;       /* generalized coordinate index; -1 if constant  */
    int32_t knot_begin;  /* first knot in mh_model.knot_x / knot_y        */
    int32_t knot_count;
    double a;
    double b;
    double scale;
    double reserved;
} mh_function;

/* One elementary joint axis (a SimTK FunctionBased mobility).  A joint is a
 * list of axes: translations are along axes fixed in the joint's parent
 * frame F; rotations are a body-fixed sequence about the joint's child
 * frame origin (Simbody MobilizedBody::FunctionBased semantics). PinJoint,
 * SliderJoint, PlanarJoint and CustomJoint all lower to this form. */
enum mh_axis_type { MH_AXIS_ROTATION = 0, MH_AXIS_TRANSLATION = 1 };
typedef struct mh_axis {
    int32_t type;
    int32_t func;        /* index into mh_model.functions                 */
    double dir[3];       /* unit axis                                      */
} mh_axis;

/* A rigid body and the joint connecting it to its parent.  Bodies must be
 * listed in topological order (parent index < own index). */
typedef struct mh_body {
    int32_t parent;      /* -1 = ground                                   */
    int32_t axis_begin;
    int32_t axis_count;  /* 0 = weld                                      */
    int32_t reserved;
    double mass;
    double com[3];       /* in body frame                                  */
    double inertia[6];   /* about COM, body frame: xx yy zz xy xz yz       */
    double R_PF[9];      /* joint parent frame F in parent body (row-major)*/
    double p_PF[3];
    double R_BM[9];      /* joint child frame M in this body               */
    double p_BM[3];
} mh_body;

/* Muscle path points (OpenSim PathPoint / ConditionalPathPoint /
 * MovingPathPoint). */
enum mh_path_point_kind { MH_PP_FIXED = 0, MH_PP_CONDITIONAL = 1, MH_PP_MOVING = 2 };
typedef struct mh_path_point {
    int32_t kind;
    int32_t body;        /* -1 = ground                                   */
    int32_t coord;       /* conditional: coordinate tested                 */
    int32_t fx, fy, fz;  /* moving: location functions (-1 = use loc[i])   */
    double loc[3];
    double range[2];     /* conditional: active when range[0]<=q<=range[1]*/
} mh_path_point;

/* DeGrooteFregly2016Muscle properties
 * (Moco/Moco/Components/DeGrooteFregly2016Muscle.{h,cpp}). */
typedef struct mh_muscle {
    int32_t point_begin;
    int32_t point_count;
    int32_t ignore_activation_dynamics;
    int32_t ignore_tendon_compliance;
    int32_t ignore_passive_fiber_force;
    int32_t tendon_dynamics_implicit;   /* tendon_compliance_dynamics_mode
                                         * "implicit" (compliant only):
                                         * the normalized tendon force
                                         * derivative is a derivative
                                         * variable and the equilibrium
                                         * FT - FM cos(alpha) an auxiliary
                                         * residual row per grid point   */
    double max_isometric_force;
    double optimal_fiber_length;
    double tendon_slack_length;
    double pennation_angle_at_optimal;
    double max_contraction_velocity;
    double activation_time_constant;
    double deactivation_time_constant;
    double fiber_damping;
    double passive_fiber_strain_at_one_norm_force;
    double tendon_strain_at_one_norm_force;
    double active_force_width_scale;
} mh_muscle;

/* Actuators, in model order; each contributes one control. */
enum mh_actuator_kind { MH_ACT_MUSCLE = 0, MH_ACT_COORDINATE = 1 };
typedef struct mh_actuator {
    int32_t kind;
    int32_t target;      /* muscle index or coordinate index               */
    double optimal_force;/* CoordinateActuator: tau = control*optimal_force*/
} mh_actuator;

/* Piecewise-polynomial table of time (data splines: ExternalForce GRF,
 * state-tracking references).  Segment s covers [breaks[s], breaks[s+1]);
 * column c value = sum_k coefs[(s*ncol + c)*(degree+1) + k] * (t-breaks[s])^k.
 * Times outside the breaks use the first/last segment polynomial. */
typedef struct mh_table {
    int32_t nseg;
    int32_t degree;
    int32_t ncol;
    int32_t break_begin; /* into mh_model.table_breaks                     */
    int32_t coef_begin;  /* into mh_model.table_coefs                      */
    int32_t reserved;
} mh_table;

/* OpenSim ExternalForce with force and point expressed in ground. */
typedef struct mh_external_force {
    int32_t body;
    int32_t table;
    int32_t force_col;   /* first of 3 columns, -1 = none                  */
    int32_t point_col;   /* first of 3 columns, -1 = body origin           */
    int32_t torque_col;  /* first of 3 columns, -1 = none                  */
    int32_t reserved;
} mh_external_force;

/* Kinematic constraints (CasOCTranscription.cpp:298-333,
 * MocoCasOCProblem.h:298-332,570-732).  OpenSim CoordinateCouplerConstraint
 * with one independent coordinate: the Simbody CoordinateCoupler of the
 * function  phi(q) = scale * f(q[f.coord]) - q[dependent]  (OpenSim's
 * CompoundFunction; f = functions[func], itself possibly a
 * MultiplierFunction).  One holonomic equation: position error phi,
 * velocity error  scale f'(q_i) u_i - u_d,  acceleration error
 * scale f'(q_i) udot_i - udot_d + scale f''(q_i) u_i u_i;  constraint
 * Jacobian row G = d phi / d q (mobility space: qdot = u); the multiplier
 * lambda adds  -G^T lambda  to the applied generalized forces (Moco negates
 * the multipliers so that Simbody's constraint forces act as applied
 * forces, MocoCasOCProblem.h:643-662). */
enum mh_constraint_kind { MH_KC_COORDINATE_COUPLER = 0 };
typedef struct mh_constraint {
    int32_t kind;        /* mh_constraint_kind                              */
    int32_t dependent;   /* coordinate index of the dependent coordinate    */
    int32_t func;        /* index into mh_model.functions (non-constant)    */
    int32_t reserved;
    double scale;        /* CoordinateCouplerConstraint scale_factor        */
} mh_constraint;

/* Wrap surfaces (ABI v5; OpenSim WrapCylinder in a body's WrapObjectSet)
 * and the PathWrap list of each muscle's GeometryPath.  The cylinder frame
 * W is fixed in the body: its z axis is the cylinder axis; a station s_W maps
 * to the body as  R_BW s_W + p_BW  (WrapObject's xyz_body_rotation, a
 * body-fixed X-Y-Z sequence, and translation).  quadrant "+x" / "-x" / "+y"
 * / "-y" constrains the wrap to that half-space of W (wrap_axis 0 / 1,
 * wrap_sign +1 / -1); "all" leaves it unconstrained (wrap_sign 0).  The
 * path algorithm is restated in oracle/oracle.c (wrap_cylinder,
 * apply_wraps) and dae_device.hpp. */
enum mh_wrap_kind { MH_WRAP_CYLINDER = 0 };
typedef struct mh_wrap_object {
    int32_t kind;        /* mh_wrap_kind                                     */
    int32_t body;        /* -1 = ground                                      */
    int32_t wrap_axis;   /* 0: x, 1: y (quadrant constraint axis)            */
    int32_t wrap_sign;   /* +1 / -1 constrained, 0 unconstrained ("all")     */
    double R_BW[9];      /* cylinder frame in the body (row-major)           */
    double p_BW[3];
    double radius;
    double length;       /* recorded; the cylinder is treated as infinite    */
} mh_wrap_object;
/* One PathWrap of a muscle, in the path's PathWrapSet order: muscles list
 * theirs contiguously (mh_muscle.wrap_begin / wrap_count below are carried
 * here as muscle + order). */
typedef struct mh_path_wrap {
    int32_t muscle;      /* muscle index (entries grouped by muscle, in order)*/
    int32_t wrap;        /* index into mh_model.wraps                         */
    int32_t range_begin; /* PathWrap range, 1-based path points; < 1 = first  */
    int32_t range_end;   /*                                       < 1 = last  */
} mh_path_wrap;

/* OpenSim SpringGeneralizedForce (ABI v8; Simulation/Model, opensim-core,
 * third-party): the generalized force  -stiffness (q - rest_length) -
 * viscosity u  on coordinate `coord`, added to the applied forces like a
 * coordinate actuator's (testMocoParameters.cpp:52-57). */
typedef struct mh_spring {
    int32_t coord;
    int32_t reserved;
    double stiffness;
    double rest_length;
    double viscosity;
} mh_spring;

typedef struct mh_model {
    int32_t nq;          /* coordinates (= speeds)                          */
    int32_t nbodies;
    int32_t naxes;
    int32_t nfunctions;
    int32_t nknots;
    int32_t nmuscles;
    int32_t npoints;
    int32_t nactuators;
    int32_t ntables;
    int32_t nbreaks;
    int32_t ncoefs;
    int32_t nexternal;
    double gravity[3];
    const mh_body* bodies;
    const mh_axis* axes;
    const mh_function* functions;
    const double* knot_x;
    const double* knot_y;
    const mh_muscle* muscles;
    const mh_path_point* points;
    const mh_actuator* actuators;
    const mh_table* tables;
    const double* table_breaks;
    const double* table_coefs;
    const mh_external_force* external;
    int32_t nconstraints;   /* enabled kinematic constraints (ABI v4)        */
    int32_t reserved_kc;
    const mh_constraint* constraints;
    int32_t nwraps;         /* wrap surfaces (ABI v5)                          */
    int32_t npathwraps;     /* PathWrap entries over all muscles               */
    const mh_wrap_object* wraps;
    const mh_path_wrap* pathwraps;
    int32_t nsprings;       /* SpringGeneralizedForce elements (ABI v8)        */
    int32_t reserved_sp;
    const mh_spring* springs;
} mh_model;

/* ------------------------------------------------------------------------ */
/* Problem (what MocoProblemRep compiles to; MocoCasOCProblem.cpp:30-251).   */
/* State order = Simbody Y order: q[0..nq), u[0..nq), then per muscle in     */
/* model order: activation (if dynamic), normalized tendon force (if         */
/* compliant).  Control order = actuator order.                              */
/* ------------------------------------------------------------------------ */

/* A NaN lower or upper means "not set" (CasOC::Bounds::isSet). */
typedef struct mh_bounds { double lower, upper; } mh_bounds;
typedef struct mh_variable_info {
    mh_bounds bounds, initial, final;
} mh_variable_info;

enum mh_goal_kind {
    MH_GOAL_CONTROL = 0,        /* MocoControlGoal                         */
    MH_GOAL_STATE_TRACKING = 1, /* MocoStateTrackingGoal                   */
    MH_GOAL_FINAL_TIME = 2,     /* MocoFinalTimeGoal                       */
    MH_GOAL_SUM_SQUARED_STATE = 3, /* MocoSumSquaredStateGoal (no reference) */
    /* minimize_implicit_auxiliary_derivatives (CasOCTranscription.cpp:534-545:
     * weight * duration * quadrature of the sum of squared implicit auxiliary
     * derivatives; MocoInverse sets it with weight 0.01, MocoInverse.cpp:
     * 106-107).  Terms index the auxiliary derivatives (0 = the first one
     * after the accelerations). */
    MH_GOAL_AUX_DERIVATIVES = 4,
    /* MocoMarkerFinalGoal (MocoMarkerFinalGoal.cpp:29-34): weight *
     * |p_G(q(tf)) - r|^2 for a point fixed on a body, at the final grid
     * point's coordinates (states required; not with prescribed
     * kinematics).  Six terms: goal_index = the body (mh_model body index,
     * -1 = ground) in each, goal_column = 0..5, goal_weight = the point's
     * location in the body frame (x, y, z) then the reference location in
     * ground (x, y, z).  An endpoint cost: no integral; its gradient is the
     * finite difference of the cost over the final coordinates (the CasADi
     * FD of the cost callback, CasOCFunction.h:38-44). */
    MH_GOAL_MARKER_FINAL = 5,
    /* minimize_lagrange_multipliers (CasOCTranscription.cpp:513-521):
     * weight * duration * quadrature of the sum of squared Lagrange
     * multipliers; terms index the multipliers.  Appended by the library
     * when mh_options.minimize_lagrange_multipliers is set (weight
     * lagrange_multiplier_weight); its gradient is exact (the reference
     * differentiates this MX expression with AD, not by finite differences). */
    MH_GOAL_LAGRANGE_MULTIPLIERS = 6
};
typedef struct mh_goal {
    int32_t kind;
    int32_t table;       /* state tracking: reference table                */
    int32_t term_begin;  /* into mh_problem.goal_index / goal_weight       */
    int32_t term_count;  /* control: #controls weighted; tracking: #states */
    int32_t exponent;    /* control goal exponent (>=2)                    */
    int32_t reserved;
    double weight;       /* MocoGoal weight                                */
} mh_goal;

/* Path constraints: MocoPathConstraint errors evaluated
 * at every mesh point (CasOCTranscription.cpp:419-433), rows placed before
 * the mesh point's residuals (flattenConstraints, CasOCTranscription.h:
 * 286-311).  A MocoControlBoundConstraint
 * (MocoControlBoundConstraint.cpp:38-146) expands, per control path in
 * order, to one equation per bound function (lower, then upper):
 *     error = control[index] - bound(t)
 * with g bounds [0, inf] (lower), [-inf, 0] (upper) or [0, 0]
 * (equality_with_lower).  bound(t) is the piecewise polynomial column
 * `column` of model table `table` (Constant: table = -1, `value`).  Each
 * equation's Jacobian row is block-dense over t0, tf and the mesh point's
 * inputs, and its values are the finite-difference quotients of the
 * path-constraint function, as for the DAE outputs. */
enum mh_path_kind { MH_PATH_CONTROL_BOUND = 0 };
typedef struct mh_path_equation {
    int32_t kind;        /* mh_path_kind                                   */
    int32_t index;       /* control index                                  */
    int32_t table;       /* bound function: model table, -1 = constant     */
    int32_t column;      /* table column                                   */
    double value;        /* constant bound (table = -1)                    */
    mh_bounds g;         /* bounds on the constraint row                   */
} mh_path_equation;

/* Endpoint constraints (CasOC endpoint constraint functions; MocoGoal in
 * Mode::EndpointConstraint, MocoGoal.h:96-137): one row of g per equation,
 * ALL of them before the first mesh point's rows (flattenConstraints,
 * CasOCTranscription.h:283-285; values CasOCTranscription.cpp:548-584).
 * An equation is a function of the Endpoint callback's inputs
 * (CasOCFunction.h:167-240): initial_time, the initial grid point's
 * states / controls / derivatives, final_time, the final grid point's.
 * Without sparsity detection its Jacobian row is dense over all of those
 * columns (ascending x order); its values are finite-difference quotients
 * of the function along each column, as for the per-point callbacks. */
enum mh_endpoint_kind {
    /* MocoInitialActivationGoal (MocoInitialActivationGoal.cpp:41-58):
     * initial control[index_a] (excitation) - initial state[index_b]
     * (activation); bounds default [0, 0] (MocoConstraintInfo.h:44-54) */
    MH_ENDPOINT_INITIAL_ACTIVATION = 0
};
typedef struct mh_endpoint_equation {
    int32_t kind;        /* mh_endpoint_kind                               */
    int32_t index_a;
    int32_t index_b;
    int32_t reserved;
    mh_bounds g;         /* bounds on the row                              */
} mh_endpoint_equation;

/* MocoParameter (ABI v8; Moco/Moco/MocoParameter.h:31-170): a scalar NLP
 * variable written into model properties before every evaluation
 * (MocoCasOCProblem.h:508-515, applyParametersToModelProperties).  The
 * parameters are the LAST block of x ("parameters", CasOCIterate.h:27-44
 * key order, CasOCTranscription.cpp:141), bounded by the MocoParameter's
 * bounds, their guess the bounds' midpoint.  One parameter may write several
 * properties (a MocoParameter over several components); each written
 * property is one target: */
enum mh_parameter_kind {
    MH_PARAM_BODY_MASS = 0,            /* Body mass                           */
    MH_PARAM_BODY_MASS_CENTER = 1,     /* Body mass_center[element]           */
    MH_PARAM_BODY_INERTIA = 2,         /* Body inertia[element], xx yy zz xy xz yz */
    MH_PARAM_SPRING_STIFFNESS = 3,     /* SpringGeneralizedForce stiffness    */
    MH_PARAM_SPRING_REST_LENGTH = 4,   /* SpringGeneralizedForce rest_length  */
    MH_PARAM_SPRING_VISCOSITY = 5,     /* SpringGeneralizedForce viscosity    */
    MH_PARAM_ACTUATOR_OPTIMAL_FORCE = 6,   /* CoordinateActuator optimal_force */
    MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE = 7 /* DGF max_isometric_force         */
};
typedef struct mh_parameter_target {
    int32_t parameter;   /* index of the NLP parameter                          */
    int32_t kind;        /* mh_parameter_kind                                   */
    int32_t index;       /* body / spring / actuator / muscle index             */
    int32_t element;     /* vector element (mass_center, inertia); else 0      */
} mh_parameter_target;

typedef struct mh_problem {
    mh_model model;
    mh_bounds time_initial;      /* bounds on initial_time                  */
    mh_bounds time_final;        /* bounds on final_time                    */
    const mh_variable_info* state_infos;   /* NS entries                    */
    const mh_variable_info* control_infos; /* NC entries                    */
    int32_t ngoals;
    int32_t nterms;
    const mh_goal* goals;
    const int32_t* goal_index;   /* control index / state index per term    */
    const int32_t* goal_column;  /* tracking: table column per term         */
    const double* goal_weight;   /* per-term weight                         */
    int32_t npath;               /* path-constraint equations per mesh point */
    int32_t reserved;
    const mh_path_equation* path;
    /* Prescribed kinematics (PositionMotion, Components/PositionMotion.cpp;
     * MocoProblemRep.cpp:74-101): prescribed_kinematics = 1 prescribes every
     * coordinate j as column kinematics_column[j] of that model table (q, and
     * its first / second time derivatives for u and udot).  The coordinate
     * values and speeds are then not NLP states (MocoProblemRep.cpp:541-555:
     * state_infos lists the auxiliary states only), there are no
     * acceleration variables, and every grid point carries nq multibody
     * residual rows (findMotionForces with the prescribed motion,
     * CasOCProblem.h:496-503).  Requires MH_DYNAMICS_IMPLICIT
     * (MocoCasADiSolver.cpp:147-151). */
    int32_t prescribed_kinematics; /* 0: none (zero-initialised default)   */
    int32_t kinematics_table;
    const int32_t* kinematics_column;
    int32_t nendpoint;           /* endpoint-constraint equations (rows 0..) */
    int32_t reserved2;
    const mh_endpoint_equation* endpoint;
    /* Kinematic constraints (model.nconstraints > 0): MocoPhase
     * multiplier_bounds (bounds of the Lagrange multipliers at every grid
     * point, initial and final alike; NaN/NaN = the reference default
     * [-1000, 1000], MocoProblem.cpp:43, MocoProblemRep.cpp:162-165) and
     * kinematic_constraint_bounds (bounds of every kinematic-constraint row;
     * NaN/NaN = the default [0, 0], MocoProblem.cpp:42). */
    mh_bounds multiplier_bounds;
    mh_bounds kinematic_constraint_bounds;
    /* MocoParameters (ABI v8, see mh_parameter_target): NP NLP variables
     * after the derivatives; every per-point callback (DAE, path
     * constraints) and the endpoint equations take them as inputs, so each
     * of those rows carries NP dense parameter columns (the last columns of
     * x), whose values are the finite-difference quotients of the callback
     * along the parameter (the property perturbed by the FD step) chained
     * through the transcription like the t0 / tf columns.  The goals of
     * mh_goal_kind do not read the model's parameterized properties: their
     * gradient along a parameter is 0.  Generic device interpreter only (a
     * generated back end folds the properties into its constant pool); no
     * sparsity detection, no batches. */
    int32_t nparameters;
    int32_t nparameter_targets;
    const mh_bounds* parameter_bounds;            /* [nparameters]             */
    const mh_parameter_target* parameter_targets; /* [nparameter_targets]      */
} mh_problem;

enum mh_scheme { MH_HERMITE_SIMPSON = 0, MH_TRAPEZOIDAL = 1 };
enum mh_fd { MH_FD_CENTRAL = 0, MH_FD_FORWARD = 1, MH_FD_BACKWARD = 2 };

typedef struct mh_options {
    int32_t num_mesh_intervals;          /* uniform mesh (CasOCSolver.h:38-42) */
    int32_t transcription;               /* mh_scheme                        */
    int32_t interpolate_control_midpoints;
    int32_t finite_difference_scheme;    /* mh_fd                            */
    double fd_step;                      /* absolute step h (<=0: 1e-8)      */
    /* Mesh-interval shard owned by this context, [interval_begin,
     * interval_end).  interval_end <= 0 means "all intervals".  A sharded
     * context evaluates the g rows / Jacobian nonzeros of its intervals
     * (CasOCTranscription.h:219-313 keeps them contiguous). */
    int32_t interval_begin;
    int32_t interval_end;
    int32_t device;                      /* HIP device ordinal               */
    /* MocoDirectCollocationSolver multibody_dynamics_mode
     * (MocoDirectCollocationSolver.h:96-153): MH_DYNAMICS_EXPLICIT, or
     * MH_DYNAMICS_IMPLICIT = generalized accelerations are NLP variables
     * ("derivatives", CasOCTranscription.cpp:134-135, bounds :222-226) and
     * the multibody equations are residual constraints at every grid point
     * (findMotionForces, MocoCasOCProblem.h:245-297;
     * CasOCTranscription.cpp:335-378; rows placed by flattenConstraints,
     * CasOCTranscription.h:219-313). */
    int32_t multibody_dynamics_mode;
    /* implicit_multibody_acceleration_bounds; {0, 0} = the reference default
     * [-1000, 1000] (MocoDirectCollocationSolver.cpp:39-40). */
    double implicit_accel_bounds[2];
    /* optim_sparsity_detection (MocoCasADiSolver.h:120-123; CasOCSolver.cpp:
     * 70-92; CasOCFunction.cpp:25-105).  NONE: every callback output
     * depends on every input of its grid point (block-dense rows).  RANDOM /
     * INITIAL_GUESS: at mh_create the DAE and path-constraint callbacks are
     * evaluated on the device at the first grid point (time = initial_time)
     * of each detection iterate, each input perturbed by +1e-5; an output
     * depends on an input iff its value changes (or is NaN), OR-ed over the
     * iterates, and Jacobian rows keep only those columns.  RANDOM uses
     * sparsity_random_count iterates (<= 0: 3) from mh_get_random_iterate on
     * uniform(-1, 1) numbers drawn from splitmix64 with seed 0, n per
     * iterate (the reference's SimTK::Random::Uniform stream is not
     * reproducible here); INITIAL_GUESS uses sparsity_guess (n doubles;
     * NULL: the bounds-midpoint guess of mh_get_initial_guess_from_bounds). */
    int32_t sparsity_detection;          /* mh_sparsity                      */
    int32_t sparsity_random_count;
    const double* sparsity_guess;
    /* GIVEN: the callback sparsity itself, as mh_get_callback_sparsity
     * returns it (e.g. detected once and reused by every shard / replica). */
    const uint8_t* sparsity_pattern;
    /* implicit_auxiliary_derivative_bounds (MocoDirectCollocationSolver.cpp:
     * 41): bounds on the derivative variables of implicit auxiliary dynamics
     * (DGF normalized tendon force with tendon_dynamics_implicit); {0, 0} =
     * the reference default [-1000, 1000]. */
    double implicit_aux_bounds[2];
    /* Kinematic constraints (ABI v4; MocoDirectCollocationSolver.cpp:29-42).
     * enforce_constraint_derivatives (reference default true): 0 = enforce
     * (position, velocity and acceleration errors as rows at every mesh
     * point; one slack "gamma" per multiplier at every mesh-interval
     * midpoint of Hermite-Simpson, whose velocity correction G^T gamma is
     * added to qdot there, CasOCTranscription.cpp:316-333), 1 = do not
     * (position errors only, no slacks).  velocity_correction_bounds: slack
     * bounds, {0, 0} = the default [-0.1, 0.1].  minimize_lagrange_multipliers
     * adds the MH_GOAL_LAGRANGE_MULTIPLIERS term with weight
     * lagrange_multiplier_weight (0 = the default 1.0); it needs kinematic
     * constraints (MocoCasOCProblem.cpp:101-107). */
    int32_t ignore_constraint_derivatives;
    int32_t minimize_lagrange_multipliers;
    double velocity_correction_bounds[2];
    double lagrange_multiplier_weight;
    /* How eval_jac_g differentiates (mh_jacobian_mode).  CALLBACK_FD (0,
     * MocoCasADiSolver): finite differences of each per-point callback
     * (fd_step, finite_difference_scheme), chained through the
     * transcription.  GLOBAL_SEEDS (1, tropter's IPOPT decorator,
     * ProblemDecorator_double.cpp:261-291): central differences of the whole
     * constraint function g along the seed directions of a column partial
     * distance-2 coloring of the Jacobian structure (GraphColoring.cpp:
     * 91-94), step sqrt(DBL_EPSILON), recovered per nonzero.  Unsharded
     * contexts only. */
    int32_t jacobian_mode;
    /* (ABI v8) The column order of that coloring (mh_coloring_order):
     * SMALLEST_LAST (0, the zero value) is ColPack's ordering as tropter
     * requests it (GraphColoring.cpp:91-94), NATURAL (1) the columns in
     * index order (ABI <= 7).  Only the seed count depends on it. */
    int32_t coloring_order;
    /* (ABI v6; v7: the values swapped) How detection decides a coupling
     * (mh_sparsity_rule).  ANY_CHANGE (0, the default of a zero-initialized
     * mh_options and of every surface above it): the reference's rule
     * (CasOCFunction.cpp:44-61: any nonzero change or NaN), under which
     * couplings that cancel to rounding level (a muscle on a coordinate it
     * does not cross) are detected or not depending on the order of the
     * floating-point operations: implementation-dependent.
     * ROBUST (1): output k depends on input j iff its change under
     * the +1e-5 perturbation is NaN or exceeds 1e-12 * the callback's
     * magnitude at the detection iterate (max(1, max over its outputs of
     * |output|)) -- a true dependency changes an output by ~1e-5 *
     * d(output) / d(input), the rounding noise of a coupling that cancels
     * stays within ~64 eps of the callback's magnitude (1.4e-14), so the
     * pattern is a property of the model: the same on the device and in any
     * other implementation. */
    int32_t sparsity_rule;
    int32_t reserved_sr;
} mh_options;

enum mh_sparsity_rule { MH_SPARSITY_RULE_ANY_CHANGE = 0, MH_SPARSITY_RULE_ROBUST = 1 };
/* ROBUST: the change, relative to the callback's magnitude, below which a
 * detection probe counts as rounding noise. */
#define MH_SPARSITY_ROBUST_TOL 1e-12

enum mh_jacobian_mode { MH_JACOBIAN_CALLBACK_FD = 0, MH_JACOBIAN_GLOBAL_SEEDS = 1 };
enum mh_coloring_order { MH_COLORING_SMALLEST_LAST = 0, MH_COLORING_NATURAL = 1 };

enum mh_sparsity {
    MH_SPARSITY_NONE = 0, MH_SPARSITY_RANDOM = 1, MH_SPARSITY_INITIAL_GUESS = 2, MH_SPARSITY_GIVEN = 3
};

enum mh_dynamics_mode { MH_DYNAMICS_EXPLICIT = 0, MH_DYNAMICS_IMPLICIT = 1 };

typedef struct mh_ctx mh_ctx;

/* Sizes of the full NLP and of this context's shard. */
typedef struct mh_nlp_info {
    int64_t n;           /* variables                                        */
    int64_t m;           /* constraints                                      */
    int64_t nnz_jac_g;   /* Jacobian nonzeros                                */
    int64_t nnz_h_lag;   /* 0: limited-memory Hessian                        */
    int64_t num_grid_points;
    int64_t num_states, num_controls;
    /* shard: rows [row_begin,row_end) and nonzeros [nnz_begin,nnz_end).
     * The head -- the endpoint-constraint rows -- precedes the first
     * interval and belongs to the shard owning it.  The tail -- the final
     * mesh point's path rows, then (implicit mode) the final grid point's
     * residual rows -- follows the last interval; the shard owning the last
     * interval owns it too.                                                */
    int64_t row_begin, row_end;
    int64_t nnz_begin, nnz_end;
} mh_nlp_info;

int mh_abi_version(void);
const char* mh_last_error(void);
/* Source hash the library was built from (tools/build_id.py: SHA-256 of
 * csrc/ and this header); lets a host detect a stale prebuilt library. */
const char* mh_build_id(void);

int mh_create(const mh_problem* problem, const mh_options* options,
        mh_ctx** ctx);
/* The sizes mh_create would give this problem and options, host only (no
 * device, no context): n, m, the grid, states / controls, the shard's rows;
 * nnz_jac_g and the shard's nonzeros of the block-dense structure (sparsity
 * detection, which needs the device, can only remove nonzeros).  Lets a
 * host size an initial-guess iterate (mh_options.sparsity_guess: n doubles)
 * before mh_create reads it. */
int mh_get_nlp_info_for(const mh_problem* problem, const mh_options* options, mh_nlp_info* info);
void mh_destroy(mh_ctx* ctx);

int mh_get_nlp_info(const mh_ctx* ctx, mh_nlp_info* info);
int mh_get_bounds(const mh_ctx* ctx, double* x_l, double* x_u, double* g_l,
        double* g_u);
int mh_get_initial_guess_from_bounds(const mh_ctx* ctx, double* x);
/* createRandomIterateWithinBounds with caller-provided uniform(-1,1) draws
 * (one per variable, in x order). */
int mh_get_random_iterate(const mh_ctx* ctx, const double* rand, double* x);
/* Full-problem structure (all rows), C_STYLE, row-major nonzero order. */
int mh_get_jac_structure(const mh_ctx* ctx, int32_t* iRow, int32_t* jCol);

/* Host-pointer evaluations.  g / values receive the FULL vectors when the
 * context is unsharded, otherwise this shard's rows / nonzeros only. */
int mh_eval_f(mh_ctx* ctx, const double* x, int new_x, double* f);
int mh_eval_grad_f(mh_ctx* ctx, const double* x, int new_x, double* grad_f);
/* The objective's partial over this context's shard (SURVEY §8(e) E2-E3:
 * the integral goals summed over the shard's own mesh intervals only --
 * CasOCTranscription.cpp:489-493 assembles the integral from the per-interval
 * quadrature -- and the endpoint goals (final time, final marker) on the
 * shard that owns the final grid point): the partials of all shards sum to
 * mh_eval_f, one all-reduce of a double.  On an unsharded context it equals
 * mh_eval_f bit for bit. */
int mh_eval_f_partial(mh_ctx* ctx, const double* x, double* f);
/* The objective's terms at x, one per goal (mh_problem.goals order: the
 * weighted value each contributes to mh_eval_f; the solution's objective
 * breakdown, MocoSolver::setSolutionStats / MocoCasADiSolver.cpp:395-402).
 * *nterms: in, the doubles terms holds; out, the number of goals (also when
 * too small: MH_ERR_INVALID).  Whole-NLP contexts; synchronous. */
int mh_eval_objective_terms(mh_ctx* ctx, const double* x, double* terms, int32_t* nterms);
/* Its gradient (n doubles): nonzero at t0 / tf and the shard's grid points
 * (the boundary point a shard shares with its neighbour carries each side's
 * share); the sum over the shards is mh_eval_grad_f (an all-reduce). */
int mh_eval_grad_f_partial(mh_ctx* ctx, const double* x, double* grad_f);
int mh_eval_g(mh_ctx* ctx, const double* x, int new_x, double* g);
int mh_eval_jac_g(mh_ctx* ctx, const double* x, int new_x, double* values);

/* Device-pointer evaluations (x, g, values in device memory of the
 * context's device), ordered on the context's stream after everything
 * enqueued on it before -- so a producer of x on that stream (see
 * mh_set_stream) needs no extra synchronization -- and synchronized before
 * returning unless the context is asynchronous (mh_set_async). */
int mh_eval_g_device(mh_ctx* ctx, const double* x_dev, double* g_dev);
int mh_eval_jac_g_device(mh_ctx* ctx, const double* x_dev,
        double* values_dev);

/* The same with IPOPT's new_x (TNLP::eval_g / eval_jac_g,
 * tropter/tropter/optimization/IPOPTSolver.cpp:383-447): new_x = 0 promises
 * that x_dev is the iterate of this context's previous mh_tnlp_eval_g_device
 * call, unchanged since (IPOPT's eval_g(new_x=true) -> eval_jac_g(new_x=false)
 * pair).  The Jacobian then depends on nothing queued after that call; with
 * MOCOHIP_OVERLAP=1 it runs on the context's auxiliary stream from that
 * point, concurrently with the eval_g kernels, and the context's stream
 * waits for it before anything queued after this call (off by default: on
 * MI355X the two cross-queue waits cost more than the overlap gains, see
 * DESIGN.md).  Results are identical to mh_eval_g_device /
 * mh_eval_jac_g_device. */
int mh_tnlp_eval_g_device(mh_ctx* ctx, const double* x_dev, int new_x, double* g_dev);
int mh_tnlp_eval_jac_g_device(mh_ctx* ctx, const double* x_dev, int new_x,
        double* values_dev);

/* eval_g and eval_jac_g at the same iterate from one device evaluation pass
 * (what an IPOPT adapter does for eval_g(new_x=true) followed by
 * eval_jac_g(new_x=false)).  Results are identical to the separate calls. */
int mh_eval_g_jac_g(mh_ctx* ctx, const double* x, double* g, double* values);
int mh_eval_g_jac_g_device(mh_ctx* ctx, const double* x_dev, double* g_dev,
        double* values_dev);

/* Order all of this context's work on `stream` (a hipStream_t of the
 * context's device, e.g. torch.cuda.current_stream().cuda_stream); NULL
 * returns to the context's own stream.  Work already enqueued on the
 * previous stream completes first. */
int mh_set_stream(mh_ctx* ctx, void* stream);
/* on != 0: mh_eval_g_device / mh_eval_jac_g_device / mh_eval_g_jac_g_device
 * return once enqueued (no host synchronization); host-pointer entries
 * always complete before returning. */
int mh_set_async(mh_ctx* ctx, int on);
/* Wait for all work enqueued on the context's stream. */
int mh_synchronize(mh_ctx* ctx);

/* Batches (BASELINE configs[4]: many IPOPT solves of one problem shape per
 * GPU, e.g. a subject / trial sweep of MocoInverse).  A batch groups 1..16
 * contexts created from structurally identical problems -- same model
 * structure (mh_model_hash up to table values), layout, options and
 * Jacobian template; each keeps its own model data (kinematics tables,
 * GRFs), iterate and outputs -- and evaluates them with one launch per
 * kernel instead of one per context (the tropter / CasADi callbacks of
 * each NLP, IPOPTSolver.cpp:417-447, for B NLPs at once).  Every batch
 * call takes B device pointers (x[b], g[b], values[b] of context b), runs
 * on the first context's stream and follows its mh_set_async setting.
 * Results are identical, bit for bit, to the contexts' own
 * mh_eval_*_device calls.  Contexts must use the task back end with the
 * fused interval kernel (generated models; no global-seed Jacobian, no
 * k_role); MH_ERR_UNSUPPORTED otherwise.  The contexts must outlive the
 * batch and must not be used concurrently with it. */
typedef struct mh_batch mh_batch;
int mh_batch_create(mh_ctx* const* ctxs, int32_t count, mh_batch** out);
void mh_batch_destroy(mh_batch* batch);
int mh_batch_eval_g_device(mh_batch* batch, const double* const* x_dev, double* const* g_dev);
int mh_batch_eval_jac_g_device(mh_batch* batch, const double* const* x_dev, double* const* v_dev);
int mh_batch_eval_g_jac_g_device(mh_batch* batch, const double* const* x_dev, double* const* g_dev,
        double* const* v_dev);
/* global_memory != 0 (default): the batched k_interval reads the group
 * results from global memory (a third of the LDS, several interval blocks
 * per CU); 0: stages them in LDS like the per-context kernel. */
int mh_batch_set_group_results_global(mh_batch* batch, int global_memory);

/* Per-point DAE probe (CasOC::Problem::calcMultibodySystemExplicit /
 * calcMultibodySystemImplicit, CasOCProblem.h:313-332) evaluated on the
 * device for npoints inputs laid out as [time, states(NS), controls(NC)]
 * (+ [udot(NQ)] in implicit mode) per point; outputs [udot(NQ), zdot(NZ)]
 * (implicit: [multibody residual(NQ), zdot(NZ)]) per point.  Used by
 * parity tests. */
int mh_eval_dae(mh_ctx* ctx, int32_t npoints, const double* inputs,
        double* outputs);

/* Identity of the device back end serving this context: the generic DAE
 * interpreter or a model-specialized (generated) kernel, the FP64 operation
 * count of one generated DAE evaluation (0 for generic), and the model hash
 * used to select it. */
int mh_get_backend(const mh_ctx* ctx, char* name, int32_t name_len,
        double* flops_per_eval, uint64_t* model_hash);
/* The back end mh_create would select for this problem and options, without
 * a device (host only): "generated:<label>" when a model-specialized back
 * end's structure (topology, joint / path / wrap / constraint wiring, the
 * zero pattern of the numbers; not their values) matches the model, else
 * "generic-<size class>". */
int mh_backend_for(const mh_problem* problem, const mh_options* options, char* name,
        int32_t name_len);
/* Kernel variants this context launches, as a space-separated list
 * ("tasks interval" = task kernels with the fused per-interval transcription
 * for the Jacobian lanes; "lane", "generic", "split", ...). */
int mh_get_backend_flags(const mh_ctx* ctx, char* flags, int32_t len);
/* The callback sparsity the Jacobian structure was built from: the NO DAE
 * outputs then the npath path equations, each a row of W = 1 + NS + NC +
 * NDV flags [time, states, controls, derivatives], then the nendpoint
 * endpoint equations, each a row of 2 W flags [initial_time, initial point
 * inputs, final_time, final point inputs] (all 1 without detection).
 * len = the capacity of `pattern` in bytes. */
int mh_get_callback_sparsity(const mh_ctx* ctx, uint8_t* pattern, int64_t len);
/* FNV-1a hash of everything the per-point DAE depends on (host only). */
int mh_model_hash(const mh_model* model, uint64_t* hash);

/* Column partial distance-2 coloring of a sparsity pattern (the seeds of
 * tropter's JacobianColoring, GraphColoring.cpp:71-120; ColPack
 * COLUMN_PARTIAL_DISTANCE_TWO): two columns share a color only if no row has
 * both.  Greedy over columns in natural order (MH_COLORING_NATURAL; see
 * mh_color_jacobian_ordered for ColPack's SMALLEST_LAST).
 * color[ncols] receives each column's seed, *ncolors the seed count.  Host
 * only (no device, no context). */
int mh_color_jacobian(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
                      const int32_t* jCol, int32_t* color, int32_t* ncolors);
/* The same with the column order chosen (mh_coloring_order).
 * MH_COLORING_SMALLEST_LAST restates ColPack's SMALLEST_LAST ordering
 * (tropter requests it, GraphColoring.cpp:91-94; Matula & Beck's
 * smallest-last order of the column intersection graph: two columns are
 * adjacent iff a row has both).  Columns sit in buckets by their number of
 * distinct adjacent columns, inserted in index order; n times the LAST column
 * of the lowest non-empty bucket is removed and placed at the end of the
 * order still free, and each of its adjacent columns not yet removed --
 * visited row by row, rows and each row's columns in the input's nonzero
 * order -- leaves its bucket (the bucket's last column takes its place) and is
 * appended to the bucket one lower.  The columns are then colored first-fit
 * in that order.  ColPack's own tie-breaking is not in the reference tree:
 * the order is this restatement's, the seed count may differ from ColPack's,
 * the recovered values cannot. */
int mh_color_jacobian_ordered(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
                              const int32_t* jCol, int32_t order, int32_t* color, int32_t* ncolors);
/* The seed of every x column (n entries) that eval_jac_g uses in
 * MH_JACOBIAN_GLOBAL_SEEDS mode (the coloring of mh_get_jac_structure). */
int mh_get_jacobian_seeds(const mh_ctx* ctx, int32_t* color, int32_t* nseeds);

/* Work of one DAE stage on this context: [0] FP64 operations executed per
 * eval_jac_g, [1] per eval_g, [2] group evaluations per eval_jac_g (task
 * back ends; 0 otherwise), [3] DAE evaluations a full re-evaluation per
 * finite-difference lane would need per eval_jac_g.  0 where unknown (the
 * generic interpreter's op count is not tracked). */
int mh_get_work(const mh_ctx* ctx, double* work4);

/* Test / debug entry (parity tests): the raw finite-difference lane outputs
 * behind mh_eval_jac_g at x (host pointers; unsharded contexts only), so a
 * checker can re-derive the Jacobian values from the same DAE outputs.
 * times[G]: each grid point's time (t0 + (tf - t0) grid_k, as the lanes
 * use it); Y[(k NO + o) S + r]: callback output o of lane r at grid point k.
 * With ND = 2 + NS + NC + NDV directions (t0, tf, then the point inputs):
 * forward / backward, S = ND + 1: lane d < ND perturbs direction d by +h /
 * -h, lane ND is unperturbed; central, S = 2 ND + 1: lanes 0..ND-1 at +h,
 * ND..2ND-1 at -h, lane 2 ND unperturbed.  A t0 / tf lane moves the time by
 * step (1 - grid_k) / step grid_k (CasOCTranscription.cpp:126-127). */
int mh_debug_jacobian_lanes(mh_ctx* ctx, const double* x, double* times,
        double* Y);

/* Benchmark entry: average device duration of each stage of eval_jac_g
 * (kind 1) or eval_g (kind 0) at the device iterate x_dev, over reps
 * (at most 500) evaluations of both stages in their call order with a HIP
 * event after each stage on the context stream (the queue stays ahead of
 * the GPU, so each figure is that kernel's own duration plus the launch gap
 * in the sequence a call runs, comparable with a rocprofv3 kernel trace).
 * ms2[0]: DAE stage, ms2[1]: transcription stage.  Results land in the
 * context's internal buffers. */
int mh_debug_time_stages(mh_ctx* ctx, const double* x_dev, int kind, int reps, double* ms2);

/* Stage timing: when on, every evaluation records HIP events between its
 * stages on the context stream and mh_last_timings reports them.  Off by
 * default (each event packet adds microseconds to a latency-bound call). */
int mh_set_timing(mh_ctx* ctx, int on);
/* Timing of the last evaluation (requires mh_set_timing(ctx, 1)), in ms:
 * [0] whole call, [1] DAE stage (k_groups + k_combine, or k_eval),
 * [2] transcription stage (k_transcribe), [3] k_groups alone (= [1] when
 * the DAE stage is one kernel). */
int mh_last_timings(const mh_ctx* ctx, double* ms4);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MOCOHIP_H */
