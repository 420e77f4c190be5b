// mh_builder.hpp — native C++ problem builder: OpenSim-level model and
// MocoProblem descriptions -> the C-ABI mh_problem (include/mocohip.h).
//
// What a C++ MocoSolver plugin needs from compileProblemRep before it can
// call mh_create: a plain C++ description of bodies, joints and their
// coordinates, DeGrooteFregly2016 muscles with their GeometryPath (fixed /
// conditional / moving path points, PathWraps over WrapCylinders),
// CoordinateActuators, ExternalForces on data tables, CoordinateCoupler
// constraints and markers, plus the problem's goals, bounds and path
// constraints, lowered with the reference's rules:
//   * coordinate order = Simbody's mobilized-body order (the multibody graph
//     grown one tree level at a time, joints in model order within a level);
//     states Y = q, u, then per muscle activation and normalized tendon force
//     (MocoUtilities.cpp:495-528 createStateVariableNamesInSystemOrder;
//     DeGrooteFregly2016Muscle.cpp:151-164); controls = actuators in
//     force-set order (MocoUtilities.cpp:557-587);
//   * default bounds (MocoProblemRep.cpp:306-444): coordinate values from the
//     coordinate range, speeds from the default speed bounds [-50, 50],
//     controls from the actuator's min/max control, activations from their
//     muscle's excitation bounds, normalized tendon force [0, 5]
//     (DeGrooteFregly2016Muscle.h:131-132);
//   * endpoint constraints of goals in endpoint-constraint mode in goal order
//     (MocoProblemRep::createEndpointConstraintNames), path constraints in
//     order (MocoControlBoundConstraint.cpp:38-118, its checks included).
// It is the same lowering as the Python host (mocohip/model.py CompiledModel,
// mocohip/problem.py ProblemRep), operation for operation, so both produce
// byte-identical mh_problem arrays (tests/test_builder.py compares the tapes).
// Data tables are given as piecewise polynomials (the GCVSpline fit of the
// samples is a third-party numerical routine; mocohip/splines.py restates it
// on the Python side).
#pragma once

#include <cmath>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "../../../include/mocohip.h"

namespace mhb {

struct Function {
    int kind = MH_FN_CONSTANT;
    std::string coord;   // empty: none
    double a = 0.0, b = 0.0, scale = 1.0;
    std::vector<double> x, y;   // SimmSpline knots
};

struct Body {
    std::string name;
    double mass = 0.0;
    double com[3] = {0, 0, 0};
    double inertia[6] = {0, 0, 0, 0, 0, 0};   // xx yy zz xy xz yz
};

struct Coordinate {
    std::string name;
    double range[2] = {-INFINITY, INFINITY};
    std::string motion_type = "rotational";
    double default_value = 0.0;
    std::string path;   // "/jointset/<joint>/<name>" unless given
};

struct Axis {
    int type = MH_AXIS_ROTATION;
    double dir[3] = {0, 0, 1};
    Function func;
};

struct Joint {
    std::string name, parent, child;
    std::vector<Coordinate> coordinates;
    std::vector<Axis> axes;
    double loc_in_parent[3] = {0, 0, 0}, orient_in_parent[3] = {0, 0, 0};
    double loc_in_child[3] = {0, 0, 0}, orient_in_child[3] = {0, 0, 0};
};

struct PathPoint {
    std::string body;
    double loc[3] = {0, 0, 0};
    int kind = MH_PP_FIXED;
    std::string coord;                  // conditional: the coordinate
    double range[2] = {0, 0};
    std::optional<Function> fx, fy, fz; // moving
    std::string name;
};

struct PathWrapRef {
    std::string wrap;
    int range_begin = -1, range_end = -1;
};

// DeGrooteFregly2016Muscle (defaults: DeGrooteFregly2016Muscle.cpp:52-63)
struct Muscle {
    std::string name, path;
    std::vector<PathPoint> points;
    double max_isometric_force = 1000.0, optimal_fiber_length = 0.1, tendon_slack_length = 0.2;
    double pennation_angle_at_optimal = 0.0, max_contraction_velocity = 10.0;
    double activation_time_constant = 0.015, deactivation_time_constant = 0.060;
    double default_activation = 0.5, default_normalized_tendon_force = 0.5;
    double active_force_width_scale = 1.0, fiber_damping = 0.0;
    double passive_fiber_strain_at_one_norm_force = 0.6, tendon_strain_at_one_norm_force = 0.049;
    bool ignore_passive_fiber_force = false, ignore_activation_dynamics = false;
    bool ignore_tendon_compliance = false;
    std::string tendon_compliance_dynamics_mode = "explicit";
    double min_control = 0.0, max_control = 1.0;
    std::vector<PathWrapRef> path_wraps;
};

struct WrapCylinder {
    std::string name, body;
    double radius = 0.0, length = 1.0;
    double xyz_body_rotation[3] = {0, 0, 0}, translation[3] = {0, 0, 0};
    std::string quadrant = "all";
    bool active = true;
};

struct CoordinateActuator {
    std::string name, coordinate;
    double optimal_force = 1.0, min_control = -INFINITY, max_control = INFINITY;
    std::string path;
};

// SpringGeneralizedForce (model.py SpringGeneralizedForce; mh_spring)
struct SpringGeneralizedForce {
    std::string name, coordinate;
    double stiffness = 0.0, rest_length = 0.0, viscosity = 0.0;
    std::string path;   // "/forceset/<name>" unless given
};

struct Marker {
    std::string name, body;
    double location[3] = {0, 0, 0};
    std::string path;
};

// A function of time as a piecewise polynomial: breaks[nseg + 1] and
// coefs[nseg][ncol][degree + 1] in ascending powers of (t - breaks[s]).
struct Table {
    std::string name;
    std::vector<std::string> columns;
    std::vector<double> breaks;
    int degree = 3;
    std::vector<double> coefs;
};

struct ExternalForce {
    std::string name, body, table;
    std::string force_identifier, point_identifier, torque_identifier;   // empty: none
};

struct CoordinateCoupler {
    std::string name, dependent;
    Function function;
    double scale_factor = 1.0;
};

class Model {
public:
    std::string name = "model";
    double gravity[3] = {0, -9.80665, 0};
    std::vector<Body> bodies;
    std::vector<Joint> joints;
    std::vector<Muscle> muscles;
    std::vector<CoordinateActuator> coordinate_actuators;
    // force-set order: (is_muscle, index into muscles / coordinate_actuators)
    std::vector<std::pair<bool, int>> actuators;
    std::vector<Table> tables;
    std::vector<ExternalForce> external_forces;
    std::vector<Marker> markers;
    std::vector<CoordinateCoupler> constraints;
    std::vector<WrapCylinder> wraps;
    std::vector<SpringGeneralizedForce> springs;

    void add_body(const Body& b) { bodies.push_back(b); }
    void add_joint(Joint j);
    void add_muscle(Muscle m);
    void add_coordinate_actuator(CoordinateActuator a);
    void add_table(const Table& t) { tables.push_back(t); }
    void add_external_force(const ExternalForce& e) { external_forces.push_back(e); }
    void add_marker(Marker m);
    void add_constraint(const CoordinateCoupler& k) { constraints.push_back(k); }
    void add_wrap(const WrapCylinder& w) { wraps.push_back(w); }
    void add_spring(SpringGeneralizedForce f);

    std::vector<const Joint*> tree_order() const;
    std::vector<const Coordinate*> coordinates() const;
    std::vector<std::string> state_names() const;
    std::vector<std::string> control_names() const;
    const Body* body(const std::string& n) const;
};

// mh_model arrays owned by value (mh_model's pointers point into them).
struct CompiledModel {
    std::vector<mh_body> bodies;
    std::vector<mh_axis> axes;
    std::vector<mh_function> functions;
    std::vector<double> knot_x, knot_y;
    std::vector<mh_muscle> muscles;
    std::vector<mh_path_point> points;
    std::vector<mh_actuator> actuators;
    std::vector<mh_table> tables;
    std::vector<double> breaks, coefs;
    std::vector<mh_external_force> external;
    std::vector<mh_constraint> constraints;
    std::vector<mh_wrap_object> wraps;
    std::vector<mh_path_wrap> pathwraps;
    std::vector<mh_spring> springs;
    std::vector<std::string> state_names, control_names;
    std::vector<std::pair<std::string, int>> body_index, qidx, table_index;
    std::vector<std::pair<std::string, std::vector<std::string>>> table_columns;
    mh_model model{};
    int index_of_body(const std::string& n) const;
    int index_of_coord(const std::string& n) const;
    int index_of_table(const std::string& n) const;
    void bind();   // (re)point model at the arrays
};

void compile_model(const Model& m, const std::vector<Table>& extra_tables, CompiledModel& out);

// ---- the problem ---------------------------------------------------------
struct Bounds {
    double lower = NAN, upper = NAN;
    bool is_set() const { return !(std::isnan(lower) || std::isnan(upper)); }
};
struct VariableInfo {
    Bounds bounds, initial, final_;
};

struct Goal {
    enum Kind { CONTROL, STATE_TRACKING, FINAL_TIME, SUM_SQUARED_STATE, INITIAL_ACTIVATION, MARKER_FINAL,
                AUX_DERIVATIVES };
    Kind kind = CONTROL;
    std::string name;
    double weight = 1.0;
    int exponent = 2;
    std::vector<std::pair<std::string, double>> weights;   // control / state weights
    std::string table;                                      // state tracking reference
    std::string mode = "endpoint_constraint";               // initial activation
    std::string point_name;                                 // marker final
    double reference_location[3] = {0, 0, 0};
};

// Bound function of MocoControlBoundConstraint: OpenSim::Constant,
// PiecewiseLinearFunction, or a GCVSpline given as its piecewise polynomial
// (x = the spline's abscissae, for the domain checks).
struct BoundFunction {
    enum Kind { NONE, CONSTANT, PIECEWISE_LINEAR, SPLINE };
    Kind kind = NONE;
    double value = 0.0;
    std::vector<double> x, y;           // piecewise linear points / spline abscissae
    std::vector<double> breaks, coefs;  // spline: coefs[nseg][1][degree + 1]
    int degree = 1;
};

struct ControlBoundConstraint {
    std::string name = "control_bound";
    std::vector<std::string> control_paths;
    BoundFunction lower, upper;
    bool equality_with_lower = false;
};

// MocoParameter (problem.py MocoParameter; MocoParameter.h:91-170):
// property_element -1 for a scalar property
struct Parameter {
    std::string name;
    std::vector<std::string> component_paths;
    std::string property_name;
    Bounds bounds;
    int property_element = -1;
};

struct Problem {
    Model model;
    std::vector<Parameter> parameters;
    Bounds time_initial, time_final;
    std::vector<std::pair<std::string, VariableInfo>> state_infos, control_infos;
    std::vector<Goal> goals;
    std::vector<ControlBoundConstraint> path_constraints;
    std::optional<Table> position_motion;   // columns: the coordinates' value paths
    Bounds default_speed_bounds{-50.0, 50.0};
    bool bound_activation_from_excitation = true;
    Bounds kinematic_constraint_bounds{0.0, 0.0};
    Bounds multiplier_bounds{-1000.0, 1000.0};
};

struct ProblemRep {
    CompiledModel cm;
    std::vector<std::string> state_names, control_names;
    std::vector<mh_variable_info> sinfo, cinfo;
    std::vector<mh_goal> goals;
    std::vector<int32_t> goal_index, goal_column;
    std::vector<double> goal_weight;
    std::vector<mh_path_equation> path;
    std::vector<mh_endpoint_equation> endpoint;
    std::vector<int32_t> kin_cols;
    std::vector<mh_bounds> parameter_bounds;
    std::vector<mh_parameter_target> parameter_targets;
    std::vector<std::string> parameter_names;
    int num_aux_residuals = 0;
    // the reference's names of the multipliers, slacks, accelerations (implicit
    // multibody dynamics) and implicit auxiliary derivatives (make_rep)
    std::vector<std::string> multiplier_names, slack_names, accel_names, aux_derivative_names;
    mh_problem problem{};
    void bind();
};

// Throws std::runtime_error with the reference's message on invalid input.
void make_rep(const Problem& p, ProblemRep& out);

// MocoHipSolver settings (mocohip/solver.py) -> mh_options.
struct SolverSettings {
    int num_mesh_intervals = 100;
    std::string transcription_scheme = "hermite-simpson";
    bool interpolate_control_midpoints = true;
    std::string optim_finite_difference_scheme = "central";
    double fd_step = 1e-8;
    int device = 0;
    std::string multibody_dynamics_mode = "explicit";
    double implicit_multibody_acceleration_bounds[2] = {-1000, 1000};
    double implicit_auxiliary_derivative_bounds[2] = {-1000, 1000};
    bool enforce_constraint_derivatives = true;
    bool minimize_lagrange_multipliers = false;
    double lagrange_multiplier_weight = 1.0;
    std::string jacobian_mode = "callback-fd";
    double velocity_correction_bounds[2] = {-0.1, 0.1};
    std::string optim_sparsity_detection = "none";
    int optim_sparsity_detection_random_count = 3;
    std::string optim_sparsity_detection_rule = "any-change";   // the reference's rule (CasOCFunction.cpp:44-61)
};
mh_options make_options(const SolverSettings& s, int interval_begin = 0, int interval_end = 0);

// The problem tape of mocohip/tape.py (version 8), byte for byte.
void write_tape(const ProblemRep& rep, const mh_options& o, const std::string& path);

// The text description written by mocohip/describe.py.
void read_description(const std::string& path, Problem& p, SolverSettings& s);

}  // namespace mhb
