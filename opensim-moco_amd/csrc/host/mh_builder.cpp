// mh_builder.cpp — see mh_builder.hpp.  Compiled with -ffp-contract=off so
// every derived number (rotation matrices, unit axes, path-bound slopes) is
// the same sequence of IEEE operations as the Python lowering.
#include "mh_builder.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace mhb {
namespace {

[[noreturn]] void fail(const std::string& msg) { throw std::runtime_error(msg); }

template <class V>
int lookup(const std::vector<std::pair<std::string, V>>& kv, const std::string& k) {
    for (size_t i = 0; i < kv.size(); ++i)
        if (kv[i].first == k) return (int)i;
    return -1;
}

// rot_x(a) @ rot_y(b) @ rot_z(c) (model.py body_fixed_xyz): OpenSim's
// body-fixed X-Y-Z frame orientation; products summed left to right.
void mm3(const double A[3][3], const double B[3][3], double C[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i][j] = (A[i][0] * B[0][j] + A[i][1] * B[1][j]) + A[i][2] * B[2][j];
}
void body_fixed_xyz(const double a[3], double* R9) {
    const double cx = std::cos(a[0]), sx = std::sin(a[0]);
    const double cy = std::cos(a[1]), sy = std::sin(a[1]);
    const double cz = std::cos(a[2]), sz = std::sin(a[2]);
    const double X[3][3] = {{1, 0, 0}, {0, cx, -sx}, {0, sx, cx}};
    const double Y[3][3] = {{cy, 0, sy}, {0, 1, 0}, {-sy, 0, cy}};
    const double Z[3][3] = {{cz, -sz, 0}, {sz, cz, 0}, {0, 0, 1}};
    double XY[3][3], R[3][3];
    mm3(X, Y, XY);
    mm3(XY, Z, R);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R9[3 * i + j] = R[i][j];
}

// WrapObject quadrant -> (wrap axis, wrap sign) (model.py quadrant_axis_sign)
void quadrant_axis_sign(std::string q, int& axis, int& sign) {
    std::string s;
    for (char ch : q)
        if (!std::isspace((unsigned char)ch)) s += (char)std::tolower((unsigned char)ch);
    if (s.empty() || s == "all") { axis = 0; sign = 0; return; }
    sign = s[0] == '-' ? -1 : 1;
    size_t k = 0;
    while (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
    const std::string ax = s.substr(k);
    if (ax != "x" && ax != "y" && ax != "z") fail("bad wrap quadrant '" + q + "'");
    if (ax == "z") fail("WrapCylinder quadrant along its axis");
    axis = ax == "x" ? 0 : 1;
}

}  // namespace

// ---- Model -----------------------------------------------------------------
void Model::add_joint(Joint j) {
    for (auto& c : j.coordinates)
        if (c.path.empty()) c.path = "/jointset/" + j.name + "/" + c.name;
    joints.push_back(std::move(j));
}
void Model::add_muscle(Muscle m) {
    if (m.path.empty()) m.path = "/forceset/" + m.name;
    muscles.push_back(std::move(m));
    actuators.emplace_back(true, (int)muscles.size() - 1);
}
void Model::add_coordinate_actuator(CoordinateActuator a) {
    if (a.path.empty()) a.path = "/forceset/" + a.name;
    coordinate_actuators.push_back(std::move(a));
    actuators.emplace_back(false, (int)coordinate_actuators.size() - 1);
}
void Model::add_spring(SpringGeneralizedForce f) {
    if (f.path.empty()) f.path = "/forceset/" + f.name;
    springs.push_back(std::move(f));
}
void Model::add_marker(Marker m) {
    if (m.path.empty()) m.path = "/markerset/" + m.name;
    for (auto& x : markers)
        if (x.path == m.path) { x = m; return; }
    markers.push_back(std::move(m));
}
const Body* Model::body(const std::string& n) const {
    for (auto& b : bodies)
        if (b.name == n) return &b;
    return nullptr;
}

// Simbody mobilized-body order: the tree grown one level at a time, joints in
// model order within a level (MultibodyGraphMaker)
std::vector<const Joint*> Model::tree_order() const {
    std::vector<const Joint*> order, remaining;
    std::vector<std::string> placed{"ground"};
    for (auto& j : joints) remaining.push_back(&j);
    auto is_placed = [&](const std::string& b) {
        return std::find(placed.begin(), placed.end(), b) != placed.end();
    };
    while (!remaining.empty()) {
        std::vector<const Joint*> level, rest;
        for (auto* j : remaining) (is_placed(j->parent) ? level : rest).push_back(j);
        if (level.empty()) fail("model graph is not a tree rooted at ground");
        for (auto* j : level) order.push_back(j);
        for (auto* j : level) placed.push_back(j->child);
        remaining = rest;
    }
    return order;
}
std::vector<const Coordinate*> Model::coordinates() const {
    std::vector<const Coordinate*> out;
    for (auto* j : tree_order())
        for (auto& c : j->coordinates) out.push_back(&c);
    return out;
}
// createStateVariableNamesInSystemOrder (MocoUtilities.cpp:495-528): q, u,
// then the muscles' auxiliary states in force-set order
std::vector<std::string> Model::state_names() const {
    std::vector<std::string> n;
    const auto qs = coordinates();
    for (auto* c : qs) n.push_back(c->path + "/value");
    for (auto* c : qs) n.push_back(c->path + "/speed");
    for (auto& m : muscles) {
        if (!m.ignore_activation_dynamics) n.push_back(m.path + "/activation");
        if (!m.ignore_tendon_compliance) n.push_back(m.path + "/normalized_tendon_force");
    }
    return n;
}
std::vector<std::string> Model::control_names() const {
    std::vector<std::string> n;
    for (auto& a : actuators) n.push_back(a.first ? muscles[a.second].path : coordinate_actuators[a.second].path);
    return n;
}

// ---- lowering to mh_model (model.py CompiledModel) --------------------------
int CompiledModel::index_of_body(const std::string& n) const {
    const int i = lookup(body_index, n);
    if (i < 0) fail("unknown body '" + n + "'");
    return body_index[i].second;
}
int CompiledModel::index_of_coord(const std::string& n) const {
    const int i = lookup(qidx, n);
    if (i < 0) fail("unknown coordinate '" + n + "'");
    return qidx[i].second;
}
int CompiledModel::index_of_table(const std::string& n) const {
    const int i = lookup(table_index, n);
    if (i < 0) fail("unknown table '" + n + "'");
    return table_index[i].second;
}

template <class T>
static T* ptr(std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

void CompiledModel::bind() {
    model.bodies = ptr(bodies);
    model.axes = ptr(axes);
    model.functions = ptr(functions);
    model.knot_x = ptr(knot_x);
    model.knot_y = ptr(knot_y);
    model.muscles = ptr(muscles);
    model.points = ptr(points);
    model.actuators = ptr(actuators);
    model.tables = ptr(tables);
    model.table_breaks = ptr(breaks);
    model.table_coefs = ptr(coefs);
    model.external = ptr(external);
    model.constraints = ptr(constraints);
    model.wraps = ptr(wraps);
    model.pathwraps = ptr(pathwraps);
    model.springs = ptr(springs);
}

void compile_model(const Model& M, const std::vector<Table>& extra_tables, CompiledModel& C) {
    C = CompiledModel();
    int qi = 0;
    for (auto* c : M.coordinates()) C.qidx.emplace_back(c->name, qi++);
    const auto joints = M.tree_order();
    C.body_index.emplace_back("ground", -1);
    for (size_t i = 0; i < joints.size(); ++i) C.body_index.emplace_back(joints[i]->child, (int)i);

    auto add_function = [&](const Function* f) -> int {
        if (!f) return -1;
        mh_function fs{};
        fs.kind = f->kind;
        fs.coord = (!f->coord.empty() && f->kind != MH_FN_CONSTANT) ? C.index_of_coord(f->coord) : -1;
        fs.a = f->a;
        fs.b = f->b;
        fs.scale = f->scale;
        if (f->kind == MH_FN_SIMMSPLINE) {
            fs.knot_begin = (int)C.knot_x.size();
            fs.knot_count = (int)f->x.size();
            C.knot_x.insert(C.knot_x.end(), f->x.begin(), f->x.end());
            C.knot_y.insert(C.knot_y.end(), f->y.begin(), f->y.end());
        }
        C.functions.push_back(fs);
        return (int)C.functions.size() - 1;
    };
    auto opt = [](const std::optional<Function>& f) { return f ? &*f : (const Function*)nullptr; };

    for (auto* j : joints) {
        const Body* B = M.body(j->child);
        if (!B) fail("joint " + j->name + ": no body " + j->child);
        mh_body b{};
        b.parent = C.index_of_body(j->parent);
        b.mass = B->mass;
        for (int k = 0; k < 3; ++k) b.com[k] = B->com[k];
        for (int k = 0; k < 6; ++k) b.inertia[k] = B->inertia[k];
        body_fixed_xyz(j->orient_in_parent, b.R_PF);
        body_fixed_xyz(j->orient_in_child, b.R_BM);
        for (int k = 0; k < 3; ++k) { b.p_PF[k] = j->loc_in_parent[k]; b.p_BM[k] = j->loc_in_child[k]; }
        b.axis_begin = (int)C.axes.size();
        for (auto& ax : j->axes) {
            mh_axis a{};
            a.type = ax.type;
            const double* d = ax.dir;
            const double n = std::sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
            for (int k = 0; k < 3; ++k) a.dir[k] = d[k] / n;
            a.func = add_function(&ax.func);
            C.axes.push_back(a);
        }
        b.axis_count = (int)C.axes.size() - b.axis_begin;
        C.bodies.push_back(b);
    }

    for (auto& m : M.muscles) {
        mh_muscle ms{};
        ms.point_begin = (int)C.points.size();
        for (auto& p : m.points) {
            mh_path_point ps{};
            ps.kind = p.kind;
            ps.body = C.index_of_body(p.body);
            for (int k = 0; k < 3; ++k) ps.loc[k] = p.loc[k];
            ps.coord = p.coord.empty() ? -1 : C.index_of_coord(p.coord);
            ps.range[0] = p.range[0];
            ps.range[1] = p.range[1];
            ps.fx = add_function(opt(p.fx));
            ps.fy = add_function(opt(p.fy));
            ps.fz = add_function(opt(p.fz));
            C.points.push_back(ps);
        }
        ms.point_count = (int)C.points.size() - ms.point_begin;
        ms.ignore_activation_dynamics = m.ignore_activation_dynamics;
        ms.ignore_tendon_compliance = m.ignore_tendon_compliance;
        ms.ignore_passive_fiber_force = m.ignore_passive_fiber_force;
        ms.tendon_dynamics_implicit = m.tendon_compliance_dynamics_mode == "implicit";
        ms.max_isometric_force = m.max_isometric_force;
        ms.optimal_fiber_length = m.optimal_fiber_length;
        ms.tendon_slack_length = m.tendon_slack_length;
        ms.pennation_angle_at_optimal = m.pennation_angle_at_optimal;
        ms.max_contraction_velocity = m.max_contraction_velocity;
        ms.activation_time_constant = m.activation_time_constant;
        ms.deactivation_time_constant = m.deactivation_time_constant;
        ms.fiber_damping = m.fiber_damping;
        ms.passive_fiber_strain_at_one_norm_force = m.passive_fiber_strain_at_one_norm_force;
        ms.tendon_strain_at_one_norm_force = m.tendon_strain_at_one_norm_force;
        ms.active_force_width_scale = m.active_force_width_scale;
        C.muscles.push_back(ms);
    }

    // wrap surfaces (model order, active ones) and the PathWraps per muscle
    std::vector<std::pair<std::string, int>> wrap_index;
    for (auto& w : M.wraps) {
        if (!w.active) continue;
        mh_wrap_object ws{};
        ws.kind = MH_WRAP_CYLINDER;
        ws.body = C.index_of_body(w.body);
        quadrant_axis_sign(w.quadrant, ws.wrap_axis, ws.wrap_sign);
        body_fixed_xyz(w.xyz_body_rotation, ws.R_BW);
        for (int k = 0; k < 3; ++k) ws.p_BW[k] = w.translation[k];
        ws.radius = w.radius;
        ws.length = w.length;
        wrap_index.emplace_back(w.name, (int)C.wraps.size());
        C.wraps.push_back(ws);
    }
    for (size_t im = 0; im < M.muscles.size(); ++im)
        for (auto& r : M.muscles[im].path_wraps) {
            const int wi = lookup(wrap_index, r.wrap);
            if (wi < 0) {
                bool inactive = false;
                for (auto& w : M.wraps) inactive |= w.name == r.wrap;
                if (inactive) continue;
                fail(M.muscles[im].name + ": unknown wrap object " + r.wrap);
            }
            mh_path_wrap pw{};
            pw.muscle = (int)im;
            pw.wrap = wrap_index[wi].second;
            pw.range_begin = r.range_begin;
            pw.range_end = r.range_end;
            C.pathwraps.push_back(pw);
        }

    for (auto& a : M.actuators) {
        mh_actuator s{};
        if (a.first) {
            s.kind = MH_ACT_MUSCLE;
            s.target = a.second;
            s.optimal_force = 1.0;
        } else {
            const auto& ca = M.coordinate_actuators[a.second];
            s.kind = MH_ACT_COORDINATE;
            s.target = C.index_of_coord(ca.coordinate);
            s.optimal_force = ca.optimal_force;
        }
        C.actuators.push_back(s);
    }

    // data tables (the model's, then the problem's) as piecewise polynomials
    std::vector<const Table*> all;
    for (auto& t : M.tables) all.push_back(&t);
    for (auto& t : extra_tables) all.push_back(&t);
    for (auto* t : all) {
        const int nseg = (int)t->breaks.size() - 1, ncol = (int)t->columns.size();
        if (nseg < 1 || (long)t->coefs.size() != (long)nseg * ncol * (t->degree + 1))
            fail("table " + t->name + ": coefficient array does not match its breaks / columns / degree");
        mh_table ts{};
        ts.nseg = nseg;
        ts.degree = t->degree;
        ts.ncol = ncol;
        ts.break_begin = (int)C.breaks.size();
        ts.coef_begin = (int)C.coefs.size();
        C.breaks.insert(C.breaks.end(), t->breaks.begin(), t->breaks.end());
        C.coefs.insert(C.coefs.end(), t->coefs.begin(), t->coefs.end());
        const int prev = lookup(C.table_index, t->name);
        if (prev >= 0) {   // a later table of the same name wins (dict semantics)
            C.table_index[prev].second = (int)C.tables.size();
            C.table_columns[prev].second = t->columns;
        } else {
            C.table_index.emplace_back(t->name, (int)C.tables.size());
            C.table_columns.emplace_back(t->name, t->columns);
        }
        C.tables.push_back(ts);
    }
    for (auto& e : M.external_forces) {
        mh_external_force es{};
        es.body = C.index_of_body(e.body);
        es.table = C.index_of_table(e.table);
        const auto& cols = C.table_columns[lookup(C.table_columns, e.table)].second;
        auto col3 = [&](const std::string& id) -> int {
            if (id.empty()) return -1;
            auto it = std::find(cols.begin(), cols.end(), id + "x");
            if (it == cols.end()) fail("external force " + e.name + ": no column " + id + "x");
            const int i = (int)(it - cols.begin());
            if (i + 2 >= (int)cols.size() || cols[i + 1] != id + "y" || cols[i + 2] != id + "z")
                fail("external force " + e.name + ": columns " + id + "x/y/z not consecutive");
            return i;
        };
        es.force_col = col3(e.force_identifier);
        es.point_col = col3(e.point_identifier);
        es.torque_col = col3(e.torque_identifier);
        C.external.push_back(es);
    }
    // kinematic constraints: their functions after every other function
    for (auto& k : M.constraints) {
        if (k.function.kind == MH_FN_CONSTANT || k.function.coord.empty())
            fail("constraint " + k.name + ": needs a function of the independent coordinate");
        mh_constraint ks{};
        ks.kind = MH_KC_COORDINATE_COUPLER;
        ks.dependent = C.index_of_coord(k.dependent);
        ks.func = add_function(&k.function);
        ks.scale = k.scale_factor;
        C.constraints.push_back(ks);
    }
    for (auto& f : M.springs) {
        mh_spring ss{};
        ss.coord = C.index_of_coord(f.coordinate);
        ss.stiffness = f.stiffness;
        ss.rest_length = f.rest_length;
        ss.viscosity = f.viscosity;
        C.springs.push_back(ss);
    }

    mh_model& mm = C.model;
    mm = mh_model{};
    mm.nq = (int)C.qidx.size();
    mm.nbodies = (int)C.bodies.size();
    mm.naxes = (int)C.axes.size();
    mm.nfunctions = (int)C.functions.size();
    mm.nknots = (int)C.knot_x.size();
    mm.nconstraints = (int)C.constraints.size();
    mm.nmuscles = (int)C.muscles.size();
    mm.npoints = (int)C.points.size();
    mm.nactuators = (int)C.actuators.size();
    mm.ntables = (int)C.tables.size();
    mm.nbreaks = (int)C.breaks.size();
    mm.ncoefs = (int)C.coefs.size();
    mm.nexternal = (int)C.external.size();
    for (int k = 0; k < 3; ++k) mm.gravity[k] = M.gravity[k];
    mm.nwraps = (int)C.wraps.size();
    mm.npathwraps = (int)C.pathwraps.size();
    mm.nsprings = (int)C.springs.size();
    C.state_names = M.state_names();
    C.control_names = M.control_names();
    C.bind();
}

// ---- MocoProblemRep (problem.py ProblemRep) ---------------------------------
void ProblemRep::bind() {
    cm.bind();
    problem.model = cm.model;
    problem.state_infos = ptr(sinfo);
    problem.control_infos = ptr(cinfo);
    problem.goals = ptr(goals);
    problem.goal_index = ptr(goal_index);
    problem.goal_column = ptr(goal_column);
    problem.goal_weight = ptr(goal_weight);
    problem.path = ptr(path);
    problem.kinematics_column = ptr(kin_cols);
    problem.endpoint = ptr(endpoint);
    problem.parameter_bounds = ptr(parameter_bounds);
    problem.parameter_targets = ptr(parameter_targets);
}

namespace {
VariableInfo& setdefault(std::vector<std::pair<std::string, VariableInfo>>& kv, const std::string& k) {
    const int i = lookup(kv, k);
    if (i >= 0) return kv[i].second;
    kv.emplace_back(k, VariableInfo());
    return kv.back().second;
}
mh_variable_info vi(const VariableInfo& v) {
    mh_variable_info o{};
    o.bounds.lower = v.bounds.lower; o.bounds.upper = v.bounds.upper;
    o.initial.lower = v.initial.lower; o.initial.upper = v.initial.upper;
    o.final.lower = v.final_.lower; o.final.upper = v.final_.upper;
    return o;
}
std::string num(double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}

// MocoControlBoundConstraint path equations (problem.py _path_equations,
// MocoControlBoundConstraint.cpp:38-118); bound functions other than
// Constant become tables appended after the model's
void path_equations(const Problem& P, std::vector<mh_path_equation>& eqs, std::vector<Table>& tables) {
    const auto names = P.model.control_names();
    auto cidx = [&](const std::string& n) {
        auto it = std::find(names.begin(), names.end(), n);
        return it == names.end() ? -1 : (int)(it - names.begin());
    };
    for (size_t ci = 0; ci < P.path_constraints.size(); ++ci) {
        const auto& pc = P.path_constraints[ci];
        const bool has_lo = pc.lower.kind != BoundFunction::NONE, has_up = pc.upper.kind != BoundFunction::NONE;
        if (!pc.control_paths.empty() && !(has_lo || has_up)) continue;   // the reference warns
        for (auto& path : pc.control_paths)
            if (cidx(path) < 0)
                fail("Control path '" + path + "' was provided but no such control exists in the model.");
        if (pc.equality_with_lower && has_up)
            fail("If equality_with_lower==true, upper bound function must not be set.");
        if (pc.equality_with_lower && !has_lo)
            fail("If equality_with_lower==true, lower bound function must be set.");
        for (const BoundFunction* f : {&pc.lower, &pc.upper}) {
            if (f->kind != BoundFunction::SPLINE || f->x.empty()) continue;
            const double lo = *std::min_element(f->x.begin(), f->x.end());
            const double hi = *std::max_element(f->x.begin(), f->x.end());
            if (lo > P.time_initial.lower)
                fail("The function's minimum domain value (" + num(lo) + ") must be less than or equal to "
                     "the minimum possible initial time (" + num(P.time_initial.lower) + ").");
            if (hi < P.time_final.upper)
                fail("The function's maximum domain value (" + num(hi) + ") must be greater than or equal "
                     "to the maximum possible final time (" + num(P.time_final.upper) + ").");
        }
        auto bound_ref = [&](const BoundFunction& f, const char* which, int& table, int& column, double& value) {
            column = 0;
            if (f.kind == BoundFunction::CONSTANT) { table = -1; value = f.value; return; }
            value = 0.0;
            const std::string name = "__path" + std::to_string(ci) + "_" + which;
            for (size_t t = 0; t < tables.size(); ++t)
                if (tables[t].name == name) { table = (int)t; return; }
            Table t;
            t.name = name;
            t.columns = {"bound"};
            if (f.kind == BoundFunction::PIECEWISE_LINEAR) {
                const size_t n = f.x.size();
                if (n < 2 || f.y.size() != n) fail("PiecewiseLinearFunction needs >= 2 increasing points");
                for (size_t i = 1; i < n; ++i)
                    if (!(f.x[i] - f.x[i - 1] > 0)) fail("PiecewiseLinearFunction needs >= 2 increasing points");
                t.breaks = f.x;
                t.degree = 1;
                for (size_t i = 0; i + 1 < n; ++i) {
                    t.coefs.push_back(f.y[i]);
                    t.coefs.push_back((f.y[i + 1] - f.y[i]) / (f.x[i + 1] - f.x[i]));
                }
            } else {
                t.breaks = f.breaks;
                t.degree = f.degree;
                t.coefs = f.coefs;
            }
            tables.push_back(t);
            table = (int)tables.size() - 1;
        };
        for (auto& path : pc.control_paths) {
            const std::pair<const char*, const BoundFunction*> which[2] = {{"lower", &pc.lower}, {"upper", &pc.upper}};
            for (auto& w : which) {
                if (w.second->kind == BoundFunction::NONE) continue;
                mh_path_equation e{};
                e.kind = MH_PATH_CONTROL_BOUND;
                e.index = cidx(path);
                bound_ref(*w.second, w.first, e.table, e.column, e.value);
                if (pc.equality_with_lower) { e.g.lower = 0.0; e.g.upper = 0.0; }
                else if (std::strcmp(w.first, "lower") == 0) { e.g.lower = 0.0; e.g.upper = INFINITY; }
                else { e.g.lower = -INFINITY; e.g.upper = 0.0; }
                eqs.push_back(e);
            }
        }
    }
}
}  // namespace

// MocoParameter::initializeOnModel (problem.py ProblemRep._parameter_targets):
// every component path names a component owning the property; vector
// properties need an element in range, scalar ones none.
static void parameter_targets(const Problem& P, const CompiledModel& C, ProblemRep& R) {
    const Model& model = P.model;
    struct Prop { const char* name; int kind; int nel; const char* owner; };
    static const Prop props[] = {
        {"mass", MH_PARAM_BODY_MASS, 0, "body"},
        {"mass_center", MH_PARAM_BODY_MASS_CENTER, 3, "body"},
        {"inertia", MH_PARAM_BODY_INERTIA, 6, "body"},
        {"stiffness", MH_PARAM_SPRING_STIFFNESS, 0, "spring"},
        {"rest_length", MH_PARAM_SPRING_REST_LENGTH, 0, "spring"},
        {"viscosity", MH_PARAM_SPRING_VISCOSITY, 0, "spring"},
        {"optimal_force", MH_PARAM_ACTUATOR_OPTIMAL_FORCE, 0, "actuator"},
        {"max_isometric_force", MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE, 0, "muscle"},
    };
    auto find = [&](const std::string& path, int& idx) -> std::string {
        std::string key = path;
        while (!key.empty() && key.back() == '/') key.pop_back();
        key = key.substr(key.find_last_of('/') == std::string::npos ? 0 : key.find_last_of('/') + 1);
        for (auto& b : model.bodies)
            if (path == b.name || path == "/bodyset/" + b.name || path == "/" + b.name) {
                idx = C.index_of_body(b.name);
                return "body";
            }
        for (size_t i = 0; i < model.springs.size(); ++i) {
            const auto& f = model.springs[i];
            if (path == f.name || path == f.path || key == f.name) { idx = (int)i; return "spring"; }
        }
        for (size_t i = 0; i < model.actuators.size(); ++i) {
            const auto& a = model.actuators[i];
            const std::string& n = a.first ? model.muscles[a.second].name : model.coordinate_actuators[a.second].name;
            const std::string& pth = a.first ? model.muscles[a.second].path : model.coordinate_actuators[a.second].path;
            if (path == n || path == pth) {
                idx = a.first ? a.second : (int)i;
                return a.first ? "muscle" : "actuator";
            }
        }
        fail("MocoParameter: no component '" + path + "' in the model");
        return "";
    };
    std::vector<std::string> names;
    for (size_t ip = 0; ip < P.parameters.size(); ++ip) {
        const Parameter& par = P.parameters[ip];
        if (std::find(names.begin(), names.end(), par.name) != names.end())
            fail("MocoParameter '" + par.name + "': duplicate name");
        names.push_back(par.name);
        if (par.component_paths.empty()) fail("MocoParameter '" + par.name + "': no component paths");
        const Prop* pr = nullptr;
        for (auto& x : props)
            if (par.property_name == x.name) pr = &x;
        if (!pr)
            fail("MocoParameter '" + par.name + "': property '" + par.property_name +
                 "' is not a parameterizable property of this build");
        int elem = 0;
        if (pr->nel) {
            if (par.property_element < 0 || par.property_element >= pr->nel)
                fail("MocoParameter '" + par.name + "': property '" + par.property_name +
                     "' needs an element in [0, " + std::to_string(pr->nel) + ")");
            elem = par.property_element;
        } else if (par.property_element >= 0) {
            fail("MocoParameter '" + par.name + "': a property element was given for the scalar property '" +
                 par.property_name + "'");
        }
        for (auto& path : par.component_paths) {
            int idx = -1;
            const std::string what = find(path, idx);
            if (what != pr->owner)
                fail("MocoParameter '" + par.name + "': component '" + path + "' (" + what +
                     ") has no property '" + par.property_name + "'");
            mh_parameter_target t{};
            t.parameter = (int32_t)ip;
            t.kind = pr->kind;
            t.index = idx;
            t.element = elem;
            R.parameter_targets.push_back(t);
        }
        mh_bounds b{};
        b.lower = par.bounds.lower;
        b.upper = par.bounds.upper;
        R.parameter_bounds.push_back(b);
        R.parameter_names.push_back(par.name);
    }
}

void make_rep(const Problem& P, ProblemRep& R) {
    R = ProblemRep();
    const Model& model = P.model;
    std::vector<mh_path_equation> path_eqs;
    std::vector<Table> extra;
    path_equations(P, path_eqs, extra);
    const std::vector<Table> bound_tables = extra;
    const bool presc = P.position_motion.has_value();
    if (presc) {
        std::vector<std::string> qpaths;
        for (auto* c : model.coordinates()) qpaths.push_back(c->path + "/value");
        if (P.position_motion->columns != qpaths)
            fail("PositionMotion: the table's columns must be the coordinates' value paths in coordinate order");
        Table t = *P.position_motion;
        t.name = "__position_motion";
        extra.push_back(t);
    }
    compile_model(model, extra, R.cm);
    for (auto& n : R.cm.state_names) {
        const bool qu = n.size() >= 6 && (n.compare(n.size() - 6, 6, "/value") == 0 ||
                                          n.compare(n.size() - 6, 6, "/speed") == 0);
        if (!(presc && qu)) R.state_names.push_back(n);
    }
    R.control_names = R.cm.control_names;
    auto sinfo = P.state_infos;
    auto cinfo = P.control_infos;
    // normalized tendon force in [0, 5] (DeGrooteFregly2016Muscle.h:131-132)
    for (auto& m : model.muscles)
        if (!m.ignore_tendon_compliance) {
            auto& info = setdefault(sinfo, m.path + "/normalized_tendon_force");
            if (!info.bounds.is_set()) info.bounds = Bounds{0.0, 5.0};
        }
    // coordinates: value from the range, speed from the default speed bounds
    // (MocoProblemRep.cpp:336-362)
    for (auto* c : model.coordinates()) {
        auto& vinfo = setdefault(sinfo, c->path + "/value");
        if (!vinfo.bounds.is_set()) vinfo.bounds = Bounds{c->range[0], c->range[1]};
        auto& sinf = setdefault(sinfo, c->path + "/speed");
        if (!sinf.bounds.is_set()) sinf.bounds = P.default_speed_bounds;
    }
    // controls from the actuators' min / max control; activation bounds from
    // the excitation's (MocoProblemRep.cpp:394-427)
    for (auto& a : model.actuators) {
        const std::string path = a.first ? model.muscles[a.second].path : model.coordinate_actuators[a.second].path;
        Bounds b0;
        {
            auto& info = setdefault(cinfo, path);
            if (!info.bounds.is_set())
                info.bounds = a.first ? Bounds{model.muscles[a.second].min_control, model.muscles[a.second].max_control}
                                      : Bounds{model.coordinate_actuators[a.second].min_control,
                                               model.coordinate_actuators[a.second].max_control};
            b0 = info.bounds;
        }
        if (P.bound_activation_from_excitation && a.first && !model.muscles[a.second].ignore_activation_dynamics) {
            auto& ai = setdefault(sinfo, path + "/activation");
            if (!ai.bounds.is_set()) ai.bounds = b0;
        }
    }
    for (auto& n : R.state_names) {
        const int i = lookup(sinfo, n);
        R.sinfo.push_back(vi(i >= 0 ? sinfo[i].second : VariableInfo()));
    }
    for (auto& n : R.control_names) {
        const int i = lookup(cinfo, n);
        R.cinfo.push_back(vi(i >= 0 ? cinfo[i].second : VariableInfo()));
    }
    auto sidx = [&](const std::string& n) {
        auto it = std::find(R.state_names.begin(), R.state_names.end(), n);
        return it == R.state_names.end() ? -1 : (int)(it - R.state_names.begin());
    };
    auto cidx = [&](const std::string& n) {
        auto it = std::find(R.control_names.begin(), R.control_names.end(), n);
        return it == R.control_names.end() ? -1 : (int)(it - R.control_names.begin());
    };
    auto weight = [](const std::vector<std::pair<std::string, double>>& w, const std::string& n) {
        for (auto& kv : w)
            if (kv.first == n) return kv.second;
        return 1.0;
    };
    auto term = [&](int i, int c, double w) {
        R.goal_index.push_back(i);
        R.goal_column.push_back(c);
        R.goal_weight.push_back(w);
    };
    // goals; endpoint-constraint-mode goals become endpoint equations in goal
    // order (MocoProblemRep::createEndpointConstraintNames)
    for (auto& g : P.goals) {
        if (g.kind == Goal::INITIAL_ACTIVATION) {
            if (g.mode != "endpoint_constraint")
                fail("MocoInitialActivationGoal in cost mode (only the endpoint-constraint default is on "
                     "the hot path)");
            for (auto& mu : model.muscles) {
                if (mu.ignore_activation_dynamics) continue;
                mh_endpoint_equation e{};
                e.kind = MH_ENDPOINT_INITIAL_ACTIVATION;
                e.index_a = cidx(mu.path);
                e.index_b = sidx(mu.path + "/activation");
                e.g.lower = 0.0;
                e.g.upper = 0.0;
                R.endpoint.push_back(e);
            }
            continue;
        }
        mh_goal gs{};
        gs.weight = g.weight;
        gs.term_begin = (int)R.goal_index.size();
        gs.table = -1;
        gs.exponent = 2;
        switch (g.kind) {
        case Goal::CONTROL:
            gs.kind = MH_GOAL_CONTROL;
            gs.exponent = g.exponent;
            if (gs.exponent < 2) fail("Exponent must be 2 or greater.");
            for (auto& n : R.control_names) {
                const double w = weight(g.weights, n);
                if (w != 0.0) term(cidx(n), -1, w);
            }
            break;
        case Goal::STATE_TRACKING: {
            gs.kind = MH_GOAL_STATE_TRACKING;
            const int ti = lookup(R.cm.table_index, g.table);
            if (ti < 0) fail("reference table " + g.table + " not in model");
            gs.table = R.cm.table_index[ti].second;
            const auto& cols = R.cm.table_columns[lookup(R.cm.table_columns, g.table)].second;
            for (size_t c = 0; c < cols.size(); ++c) {
                if (sidx(cols[c]) < 0) fail("State reference '" + cols[c] + "' unrecognized.");
                term(sidx(cols[c]), (int)c, weight(g.weights, cols[c]));
            }
            break;
        }
        case Goal::FINAL_TIME:
            gs.kind = MH_GOAL_FINAL_TIME;
            break;
        case Goal::MARKER_FINAL: {
            if (presc)
                fail("MocoMarkerFinalGoal with prescribed kinematics (the final coordinates are not NLP states)");
            const Marker* mk = nullptr;
            for (auto& x : model.markers)
                if (x.path == g.point_name) mk = &x;
            if (!mk) fail("MocoMarkerFinalGoal: no point '" + g.point_name + "' in the model");
            const int body = R.cm.index_of_body(mk->body);
            gs.kind = MH_GOAL_MARKER_FINAL;
            for (int c = 0; c < 3; ++c) term(body, c, mk->location[c]);
            for (int c = 0; c < 3; ++c) term(body, 3 + c, g.reference_location[c]);
            break;
        }
        case Goal::AUX_DERIVATIVES: {
            gs.kind = MH_GOAL_AUX_DERIVATIVES;
            int naux = 0;
            for (auto& m : model.muscles)
                naux += !m.ignore_tendon_compliance && m.tendon_compliance_dynamics_mode == "implicit";
            for (int k = 0; k < naux; ++k) term(k, -1, 1.0);
            break;
        }
        case Goal::SUM_SQUARED_STATE:
            gs.kind = MH_GOAL_SUM_SQUARED_STATE;
            for (auto& n : R.state_names) {
                const double w = weight(g.weights, n);
                if (w != 0.0) term(sidx(n), -1, w);
            }
            break;
        default:
            fail("unsupported goal");
        }
        gs.term_count = (int)R.goal_index.size() - gs.term_begin;
        R.goals.push_back(gs);
    }
    for (auto& e : path_eqs)
        if (e.table >= 0) e.table = R.cm.index_of_table(bound_tables[e.table].name);
    R.path = path_eqs;
    mh_problem& p = R.problem;
    p = mh_problem{};
    p.time_initial.lower = P.time_initial.lower;
    p.time_initial.upper = P.time_initial.upper;
    p.time_final.lower = P.time_final.lower;
    p.time_final.upper = P.time_final.upper;
    p.ngoals = (int)R.goals.size();
    p.nterms = (int)R.goal_index.size();
    p.prescribed_kinematics = 0;
    if (presc) {
        p.prescribed_kinematics = 1;
        p.kinematics_table = R.cm.index_of_table("__position_motion");
        for (int q = 0; q < R.cm.model.nq; ++q) R.kin_cols.push_back(q);
    }
    p.npath = (int)R.path.size();
    p.nendpoint = (int)R.endpoint.size();
    parameter_targets(P, R.cm, R);
    p.nparameters = (int)R.parameter_bounds.size();
    p.nparameter_targets = (int)R.parameter_targets.size();
    p.multiplier_bounds.lower = P.multiplier_bounds.lower;
    p.multiplier_bounds.upper = P.multiplier_bounds.upper;
    p.kinematic_constraint_bounds.lower = P.kinematic_constraint_bounds.lower;
    p.kinematic_constraint_bounds.upper = P.kinematic_constraint_bounds.upper;
    for (auto& m : model.muscles)
        R.num_aux_residuals += !m.ignore_tendon_compliance && m.tendon_compliance_dynamics_mode == "implicit";
    // the reference's names of the other variable blocks (problem.py
    // ProblemRep): multipliers lambda_cid<c>_p0 after the Simbody
    // ConstraintIndex c -- every Coordinate owns a (disabled) lock constraint
    // ahead of the ConstraintSet, so the enabled couplers are c = ncoord + i
    // (MocoProblemRep.cpp:202-230) --, slacks gamma_cid<c>_p0
    // (MocoCasOCProblem.cpp:186-201), accelerations <coordinate>/accel
    // (CasOCProblem.h:363-377), implicit auxiliary derivatives
    // <muscle>/implicitderiv_normalized_tendon_force (MocoProblemRep.cpp:445-460)
    const int ncoord = (int)model.coordinates().size();
    R.multiplier_names.clear();
    R.slack_names.clear();
    for (size_t i = 0; i < model.constraints.size(); ++i) {
        R.multiplier_names.push_back("lambda_cid" + std::to_string(ncoord + (int)i) + "_p0");
        R.slack_names.push_back("gamma_cid" + std::to_string(ncoord + (int)i) + "_p0");
    }
    R.accel_names.clear();
    for (auto& n : R.state_names)
        if (n.size() >= 6 && n.compare(n.size() - 6, 6, "/speed") == 0)
            R.accel_names.push_back(n.substr(0, n.size() - 5) + "accel");
    R.aux_derivative_names.clear();
    for (auto& m : model.muscles)
        if (!m.ignore_tendon_compliance && m.tendon_compliance_dynamics_mode == "implicit")
            R.aux_derivative_names.push_back(m.path + "/implicitderiv_normalized_tendon_force");
    R.bind();
}

// ---- solver settings (solver.py MocoHipSolver.options) ----------------------
mh_options make_options(const SolverSettings& s, int interval_begin, int interval_end) {
    mh_options o;
    std::memset(&o, 0, sizeof o);
    if (s.transcription_scheme == "hermite-simpson") o.transcription = MH_HERMITE_SIMPSON;
    else if (s.transcription_scheme == "trapezoidal") o.transcription = MH_TRAPEZOIDAL;
    else fail("transcription_scheme '" + s.transcription_scheme + "' not in {'trapezoidal', 'hermite-simpson'}");
    if (s.optim_finite_difference_scheme == "central") o.finite_difference_scheme = MH_FD_CENTRAL;
    else if (s.optim_finite_difference_scheme == "forward") o.finite_difference_scheme = MH_FD_FORWARD;
    else if (s.optim_finite_difference_scheme == "backward") o.finite_difference_scheme = MH_FD_BACKWARD;
    else fail("optim_finite_difference_scheme must be one of central, forward, backward");
    if (s.multibody_dynamics_mode == "explicit") o.multibody_dynamics_mode = MH_DYNAMICS_EXPLICIT;
    else if (s.multibody_dynamics_mode == "implicit") o.multibody_dynamics_mode = MH_DYNAMICS_IMPLICIT;
    else fail("multibody_dynamics_mode must be 'explicit' or 'implicit'");
    if (s.optim_sparsity_detection == "none") o.sparsity_detection = MH_SPARSITY_NONE;
    else if (s.optim_sparsity_detection == "random") o.sparsity_detection = MH_SPARSITY_RANDOM;
    // "initial-guess" (CasOCSolver.cpp:74-76): the caller points
    // o.sparsity_guess at the guess iterate (null: the bounds midpoint)
    else if (s.optim_sparsity_detection == "initial-guess") o.sparsity_detection = MH_SPARSITY_INITIAL_GUESS;
    else fail("optim_sparsity_detection must be 'none', 'random' or 'initial-guess'");
    o.num_mesh_intervals = s.num_mesh_intervals;
    o.interpolate_control_midpoints = s.interpolate_control_midpoints;
    o.fd_step = s.fd_step;
    o.interval_begin = interval_begin;
    o.interval_end = interval_end;
    o.device = s.device;
    o.implicit_accel_bounds[0] = s.implicit_multibody_acceleration_bounds[0];
    o.implicit_accel_bounds[1] = s.implicit_multibody_acceleration_bounds[1];
    o.implicit_aux_bounds[0] = s.implicit_auxiliary_derivative_bounds[0];
    o.implicit_aux_bounds[1] = s.implicit_auxiliary_derivative_bounds[1];
    o.ignore_constraint_derivatives = s.enforce_constraint_derivatives ? 0 : 1;
    o.minimize_lagrange_multipliers = s.minimize_lagrange_multipliers;
    o.lagrange_multiplier_weight = s.lagrange_multiplier_weight;
    if (s.jacobian_mode == "callback-fd") o.jacobian_mode = MH_JACOBIAN_CALLBACK_FD;
    else if (s.jacobian_mode == "global-seeds") o.jacobian_mode = MH_JACOBIAN_GLOBAL_SEEDS;
    else fail("jacobian_mode must be 'callback-fd' or 'global-seeds'");
    o.velocity_correction_bounds[0] = s.velocity_correction_bounds[0];
    o.velocity_correction_bounds[1] = s.velocity_correction_bounds[1];
    o.sparsity_random_count = s.optim_sparsity_detection_random_count;
    if (s.optim_sparsity_detection_rule == "robust") o.sparsity_rule = MH_SPARSITY_RULE_ROBUST;
    else if (s.optim_sparsity_detection_rule == "any-change") o.sparsity_rule = MH_SPARSITY_RULE_ANY_CHANGE;
    else fail("optim_sparsity_detection_rule must be 'robust' or 'any-change'");
    return o;
}

// ---- the tape (mocohip/tape.py write_tape, version 8) -----------------------
namespace {
struct Out {
    std::string b;
    template <class T>
    void pod(const T& v) { b.append(reinterpret_cast<const char*>(&v), sizeof v); }
    void bytes(const void* p, size_t n) { if (n) b.append(reinterpret_cast<const char*>(p), n); }
    template <class T>
    void blob(const T* p, long count) {
        const int64_t n = (p && count > 0) ? (int64_t)(sizeof(T) * count) : 0;
        pod(n);
        bytes(p, (size_t)n);
    }
};
}  // namespace

void write_tape(const ProblemRep& R, const mh_options& o0, const std::string& path) {
    const mh_problem& p = R.problem;
    const mh_model& m = p.model;
    const int32_t ns = (int32_t)R.state_names.size(), nc = (int32_t)R.control_names.size();
    mh_options o;
    std::memcpy(&o, &o0, sizeof o);   // padding included (tape.py writes the struct's bytes)
    o.sparsity_guess = nullptr;
    o.sparsity_pattern = nullptr;
    Out w;
    w.bytes("MHTAPE01", 8);
    const int32_t head[3] = {8, ns, nc};
    w.bytes(head, sizeof head);
    w.pod(o);
    const int32_t counts[12] = {m.nq, m.nbodies, m.naxes, m.nfunctions, m.nknots, m.nmuscles,
                                m.npoints, m.nactuators, m.ntables, m.nbreaks, m.ncoefs, m.nexternal};
    w.bytes(counts, sizeof counts);
    w.bytes(m.gravity, sizeof m.gravity);
    w.pod(p.time_initial);
    w.pod(p.time_final);
    const int32_t ng[2] = {p.ngoals, p.nterms};
    w.bytes(ng, sizeof ng);
    w.blob(m.bodies, m.nbodies);
    w.blob(m.axes, m.naxes);
    w.blob(m.functions, m.nfunctions);
    w.blob(m.knot_x, m.nknots);
    w.blob(m.knot_y, m.nknots);
    w.blob(m.muscles, m.nmuscles);
    w.blob(m.points, m.npoints);
    w.blob(m.actuators, m.nactuators);
    w.blob(m.tables, m.ntables);
    w.blob(m.table_breaks, m.nbreaks);
    w.blob(m.table_coefs, m.ncoefs);
    w.blob(m.external, m.nexternal);
    w.blob(p.state_infos, ns);
    w.blob(p.control_infos, nc);
    w.blob(p.goals, p.ngoals);
    w.blob(p.goal_index, p.nterms);
    w.blob(p.goal_column, p.nterms);
    w.blob(p.goal_weight, p.nterms);
    w.pod(p.npath);
    w.blob(p.path, p.npath);
    w.pod((int64_t)0);   // no sparsity guess
    w.pod((int64_t)0);   // no given pattern
    const int32_t pk[2] = {p.prescribed_kinematics, p.kinematics_table};
    w.bytes(pk, sizeof pk);
    w.blob(p.prescribed_kinematics ? p.kinematics_column : (const int32_t*)nullptr, m.nq);
    w.pod(p.nendpoint);
    w.blob(p.endpoint, p.nendpoint);
    w.pod(m.nconstraints);
    w.blob(m.constraints, m.nconstraints);
    w.pod(p.multiplier_bounds);
    w.pod(p.kinematic_constraint_bounds);
    w.pod(m.nwraps);
    w.blob(m.wraps, m.nwraps);
    w.pod(m.npathwraps);
    w.blob(m.pathwraps, m.npathwraps);
    w.pod(m.nsprings);
    w.blob(m.springs, m.nsprings);
    w.pod(p.nparameters);
    w.blob(p.parameter_bounds, p.nparameters);
    w.pod(p.nparameter_targets);
    w.blob(p.parameter_targets, p.nparameter_targets);
    std::ofstream f(path, std::ios::binary);
    if (!f) fail("cannot write " + path);
    f.write(w.b.data(), (std::streamsize)w.b.size());
    if (!f) fail("write failed: " + path);
}

// ---- the description (mocohip/describe.py) ----------------------------------
namespace {
struct Tok {
    std::istringstream in;
    std::string last;
    explicit Tok(const std::string& text) : in(text) {}
    std::string s() {
        if (!(in >> last)) fail("description: unexpected end");
        return last == "~" ? std::string() : last;
    }
    std::string word() {
        if (!(in >> last)) fail("description: unexpected end");
        return last;
    }
    double d() {
        const std::string t = word();
        char* end = nullptr;
        const double v = std::strtod(t.c_str(), &end);
        if (!end || *end) fail("description: bad number '" + t + "'");
        return v;
    }
    long i() {
        const std::string t = word();
        char* end = nullptr;
        const long v = std::strtol(t.c_str(), &end, 10);
        if (!end || *end) fail("description: bad integer '" + t + "'");
        return v;
    }
    void d3(double* v, int n = 3) { for (int k = 0; k < n; ++k) v[k] = d(); }
    std::vector<double> dv(long n) {
        std::vector<double> v((size_t)n);
        for (auto& x : v) x = d();
        return v;
    }
};

std::optional<Function> read_fn(Tok& t) {
    const std::string tag = t.word();
    if (tag == "F-") return std::nullopt;
    if (tag != "F") fail("description: expected a function, got '" + tag + "'");
    Function f;
    f.kind = (int)t.i();
    f.coord = t.s();
    f.a = t.d();
    f.b = t.d();
    f.scale = t.d();
    const long n = t.i();
    f.x = t.dv(n);
    f.y = t.dv(n);
    return f;
}

Table read_table(Tok& t) {
    Table tb;
    tb.name = t.s();
    const long nc = t.i();
    for (long c = 0; c < nc; ++c) tb.columns.push_back(t.s());
    tb.breaks = t.dv(t.i());
    tb.degree = (int)t.i();
    tb.coefs = t.dv((long)(tb.breaks.size() - 1) * nc * (tb.degree + 1));
    return tb;
}

Bounds read_bounds(Tok& t) {
    Bounds b;
    b.lower = t.d();
    b.upper = t.d();
    return b;
}

BoundFunction read_bound_fn(Tok& t) {
    BoundFunction f;
    const std::string k = t.word();
    if (k == "none") return f;
    if (k == "const") { f.kind = BoundFunction::CONSTANT; f.value = t.d(); return f; }
    if (k == "pwl") {
        f.kind = BoundFunction::PIECEWISE_LINEAR;
        const long n = t.i();
        f.x = t.dv(n);
        f.y = t.dv(n);
        return f;
    }
    if (k == "spline") {
        f.kind = BoundFunction::SPLINE;
        f.x = t.dv(t.i());
        f.breaks = t.dv(t.i());
        f.degree = (int)t.i();
        f.coefs = t.dv((long)(f.breaks.size() - 1) * (f.degree + 1));
        return f;
    }
    fail("description: bad bound function '" + k + "'");
}

std::vector<std::pair<std::string, double>> read_weights(Tok& t) {
    std::vector<std::pair<std::string, double>> w;
    const long n = t.i();
    for (long k = 0; k < n; ++k) {
        const std::string name = t.s();
        w.emplace_back(name, t.d());
    }
    return w;
}
}  // namespace

void read_description(const std::string& path, Problem& P, SolverSettings& S) {
    std::ifstream f(path);
    if (!f) fail("cannot read " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    Tok t(ss.str());
    if (t.word() != "mhdesc" || t.i() != 1) fail("not a version-1 mhdesc description");
    P = Problem();
    Model& M = P.model;
    for (;;) {
        const std::string rec = t.word();
        if (rec == "end") break;
        if (rec == "model") {
            M.name = t.s();
            t.d3(M.gravity);
        } else if (rec == "body") {
            Body b;
            b.name = t.s();
            b.mass = t.d();
            t.d3(b.com);
            t.d3(b.inertia, 6);
            M.add_body(b);
        } else if (rec == "joint") {
            Joint j;
            j.name = t.s();
            j.parent = t.s();
            j.child = t.s();
            t.d3(j.loc_in_parent);
            t.d3(j.orient_in_parent);
            t.d3(j.loc_in_child);
            t.d3(j.orient_in_child);
            const long nco = t.i(), nax = t.i();
            for (long k = 0; k < nco; ++k) {
                if (t.word() != "coord") fail("description: expected coord");
                Coordinate c;
                c.name = t.s();
                t.d3(c.range, 2);
                c.motion_type = t.s();
                c.default_value = t.d();
                c.path = t.s();
                j.coordinates.push_back(c);
            }
            for (long k = 0; k < nax; ++k) {
                if (t.word() != "axis") fail("description: expected axis");
                Axis a;
                a.type = (int)t.i();
                t.d3(a.dir);
                auto fn = read_fn(t);
                if (!fn) fail("description: an axis needs a function");
                a.func = *fn;
                j.axes.push_back(a);
            }
            M.add_joint(j);
        } else if (rec == "wrap") {
            WrapCylinder w;
            w.name = t.s();
            w.body = t.s();
            w.radius = t.d();
            w.length = t.d();
            t.d3(w.xyz_body_rotation);
            t.d3(w.translation);
            w.quadrant = t.s();
            w.active = t.i() != 0;
            M.add_wrap(w);
        } else if (rec == "muscle") {
            Muscle m;
            m.name = t.s();
            m.path = t.s();
            const long npt = t.i();
            double* params[] = {&m.max_isometric_force, &m.optimal_fiber_length, &m.tendon_slack_length,
                                &m.pennation_angle_at_optimal, &m.max_contraction_velocity,
                                &m.activation_time_constant, &m.deactivation_time_constant,
                                &m.default_activation, &m.default_normalized_tendon_force,
                                &m.active_force_width_scale, &m.fiber_damping,
                                &m.passive_fiber_strain_at_one_norm_force, &m.tendon_strain_at_one_norm_force};
            for (double* p : params) *p = t.d();
            m.ignore_passive_fiber_force = t.i() != 0;
            m.ignore_activation_dynamics = t.i() != 0;
            m.ignore_tendon_compliance = t.i() != 0;
            m.tendon_compliance_dynamics_mode = t.s();
            m.min_control = t.d();
            m.max_control = t.d();
            const long nw = t.i();
            for (long k = 0; k < nw; ++k) {
                PathWrapRef r;
                r.wrap = t.s();
                r.range_begin = (int)t.i();
                r.range_end = (int)t.i();
                m.path_wraps.push_back(r);
            }
            for (long k = 0; k < npt; ++k) {
                if (t.word() != "point") fail("description: expected point");
                PathPoint p;
                p.body = t.s();
                t.d3(p.loc);
                p.kind = (int)t.i();
                p.coord = t.s();
                t.d3(p.range, 2);
                p.fx = read_fn(t);
                p.fy = read_fn(t);
                p.fz = read_fn(t);
                p.name = t.s();
                m.points.push_back(p);
            }
            M.add_muscle(m);
        } else if (rec == "coordact") {
            CoordinateActuator a;
            a.name = t.s();
            a.coordinate = t.s();
            a.optimal_force = t.d();
            a.min_control = t.d();
            a.max_control = t.d();
            a.path = t.s();
            M.add_coordinate_actuator(a);
        } else if (rec == "spring") {
            SpringGeneralizedForce f;
            f.name = t.s();
            f.coordinate = t.s();
            f.stiffness = t.d();
            f.rest_length = t.d();
            f.viscosity = t.d();
            f.path = t.s();
            M.add_spring(f);
        } else if (rec == "marker") {
            Marker mk;
            mk.name = t.s();
            mk.body = t.s();
            t.d3(mk.location);
            mk.path = t.s();
            M.add_marker(mk);
        } else if (rec == "constraint") {
            CoordinateCoupler k;
            k.name = t.s();
            k.dependent = t.s();
            auto fn = read_fn(t);
            if (!fn) fail("description: a constraint needs a function");
            k.function = *fn;
            k.scale_factor = t.d();
            M.add_constraint(k);
        } else if (rec == "table") {
            M.add_table(read_table(t));
        } else if (rec == "extforce") {
            ExternalForce e;
            e.name = t.s();
            e.body = t.s();
            e.table = t.s();
            e.force_identifier = t.s();
            e.point_identifier = t.s();
            e.torque_identifier = t.s();
            M.add_external_force(e);
        } else if (rec == "problem") {
            P.time_initial = read_bounds(t);
            P.time_final = read_bounds(t);
            P.default_speed_bounds = read_bounds(t);
            P.bound_activation_from_excitation = t.i() != 0;
            P.kinematic_constraint_bounds = read_bounds(t);
            P.multiplier_bounds = read_bounds(t);
        } else if (rec == "stateinfo" || rec == "controlinfo") {
            const std::string n = t.s();
            VariableInfo v;
            v.bounds = read_bounds(t);
            v.initial = read_bounds(t);
            v.final_ = read_bounds(t);
            (rec == "stateinfo" ? P.state_infos : P.control_infos).emplace_back(n, v);
        } else if (rec == "goal") {
            const std::string kind = t.word();
            Goal g;
            if (kind == "control") {
                g.kind = Goal::CONTROL;
                g.name = t.s(); g.weight = t.d(); g.exponent = (int)t.i(); g.weights = read_weights(t);
            } else if (kind == "state_tracking") {
                g.kind = Goal::STATE_TRACKING;
                g.name = t.s(); g.weight = t.d(); g.table = t.s(); g.weights = read_weights(t);
            } else if (kind == "final_time") {
                g.kind = Goal::FINAL_TIME;
                g.name = t.s(); g.weight = t.d();
            } else if (kind == "sum_squared_state") {
                g.kind = Goal::SUM_SQUARED_STATE;
                g.name = t.s(); g.weight = t.d(); g.weights = read_weights(t);
            } else if (kind == "initial_activation") {
                g.kind = Goal::INITIAL_ACTIVATION;
                g.name = t.s(); g.mode = t.s(); g.weight = t.d();
            } else if (kind == "marker_final") {
                g.kind = Goal::MARKER_FINAL;
                g.name = t.s(); g.weight = t.d(); g.point_name = t.s(); t.d3(g.reference_location);
            } else if (kind == "aux_derivatives") {
                g.kind = Goal::AUX_DERIVATIVES;
                g.name = t.s(); g.weight = t.d();
            } else {
                fail("description: unknown goal kind '" + kind + "'");
            }
            P.goals.push_back(g);
        } else if (rec == "pathcon") {
            ControlBoundConstraint pc;
            pc.name = t.s();
            const long n = t.i();
            for (long k = 0; k < n; ++k) pc.control_paths.push_back(t.s());
            pc.lower = read_bound_fn(t);
            pc.upper = read_bound_fn(t);
            pc.equality_with_lower = t.i() != 0;
            P.path_constraints.push_back(pc);
        } else if (rec == "parameter") {
            Parameter par;
            par.name = t.s();
            par.property_name = t.s();
            par.property_element = (int)t.i();
            par.bounds = read_bounds(t);
            const long n = t.i();
            for (long k = 0; k < n; ++k) par.component_paths.push_back(t.s());
            P.parameters.push_back(par);
        } else if (rec == "position_motion") {
            if (t.word() != "table") fail("description: position_motion needs a table");
            P.position_motion = read_table(t);
        } else if (rec == "solver") {
            S.num_mesh_intervals = (int)t.i();
            S.transcription_scheme = t.s();
            S.interpolate_control_midpoints = t.i() != 0;
            S.optim_finite_difference_scheme = t.s();
            S.fd_step = t.d();
            S.device = (int)t.i();
            S.multibody_dynamics_mode = t.s();
            t.d3(S.implicit_multibody_acceleration_bounds, 2);
            t.d3(S.implicit_auxiliary_derivative_bounds, 2);
            S.enforce_constraint_derivatives = t.i() != 0;
            S.minimize_lagrange_multipliers = t.i() != 0;
            S.lagrange_multiplier_weight = t.d();
            S.jacobian_mode = t.s();
            t.d3(S.velocity_correction_bounds, 2);
            S.optim_sparsity_detection = t.s();
            S.optim_sparsity_detection_random_count = (int)t.i();
            S.optim_sparsity_detection_rule = t.s();
        } else {
            fail("description: unknown record '" + rec + "'");
        }
    }
}

}  // namespace mhb
