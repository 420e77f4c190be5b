/* MocoHipSolver.cpp — see MocoHipSolver.h.  NOT compiled in this repository
 * (OpenSim and Ipopt are absent from the image); written
 * against opensim-core b0222c2's public headers and Ipopt 3.12.8.
 *
 * Pieces, each mirroring the reference function it replaces:
 *   compileProblemRep    the Model / MocoProblemRep walk (MocoProblemRep.h:
 *                        69-116) into mhb::Problem: the same rules as the
 *                        Python lowering of .osim files (mocohip/osim.py,
 *                        model.py, problem.py), whose tapes the C++ builder
 *                        reproduces byte for byte (tests/test_builder.py);
 *   solveImpl            MocoCasADiSolver::solveImpl (MocoCasADiSolver.cpp:
 *                        312-415): guess -> iterate, the NLP on the GPU
 *                        through the C ABI, Ipopt over it (mh_ipopt_tnlp.hpp),
 *                        the iterate back to a MocoSolution, setSolutionStats
 *                        (MocoSolver.h:97-102).
 */
#include "MocoHipSolver.h"

#include <OpenSim/Actuators/CoordinateActuator.h>
#include <OpenSim/Actuators/SpringGeneralizedForce.h>
#include <OpenSim/Common/Constant.h>
#include <OpenSim/Common/GCVSpline.h>
#include <OpenSim/Common/GCVSplineSet.h>
#include <OpenSim/Common/LinearFunction.h>
#include <OpenSim/Common/MultiplierFunction.h>
#include <OpenSim/Common/PiecewiseLinearFunction.h>
#include <OpenSim/Common/SimmSpline.h>
#include <OpenSim/Common/Stopwatch.h>
#include <OpenSim/Moco/Components/DeGrooteFregly2016Muscle.h>
#include <OpenSim/Moco/Components/PositionMotion.h>
#include <OpenSim/Moco/MocoGoal/MocoControlGoal.h>
#include <OpenSim/Moco/MocoGoal/MocoInitialActivationGoal.h>
#include <OpenSim/Moco/MocoGoal/MocoMarkerFinalGoal.h>
#include <OpenSim/Moco/MocoGoal/MocoStateTrackingGoal.h>
#include <OpenSim/Moco/MocoGoal/MocoSumSquaredStateGoal.h>
#include <OpenSim/Moco/MocoGoal/MocoGoal.h>
#include <OpenSim/Moco/MocoControlBoundConstraint.h>
#include <OpenSim/Moco/MocoProblemRep.h>
#include <OpenSim/Moco/MocoUtilities.h>
#include <OpenSim/Simulation/Model/ExternalForce.h>
#include <OpenSim/Simulation/Model/Model.h>
#include <OpenSim/Simulation/Model/PhysicalOffsetFrame.h>
#include <OpenSim/Simulation/SimbodyEngine/CoordinateCouplerConstraint.h>
#include <OpenSim/Simulation/SimbodyEngine/CustomJoint.h>
#include <OpenSim/Simulation/SimbodyEngine/PinJoint.h>
#include <OpenSim/Simulation/SimbodyEngine/SliderJoint.h>
#include <OpenSim/Simulation/SimbodyEngine/WeldJoint.h>
#include <OpenSim/Simulation/Wrap/PathWrap.h>
#include <OpenSim/Simulation/Wrap/WrapCylinder.h>
#include <OpenSim/Simulation/Model/ConditionalPathPoint.h>
#include <OpenSim/Simulation/Model/MovingPathPoint.h>

#include "mh_ipopt_tnlp.hpp"
#include "mh_trajectory.hpp"

using namespace OpenSim;

namespace {

// ---- functions -------------------------------------------------------------
// OpenSim functions of one coordinate -> mhb::Function (osim.py
// parse_function): Constant, LinearFunction, SimmSpline, and a
// MultiplierFunction scaling either.
mhb::Function toFunction(const Function& f, const std::string& coord) {
    mhb::Function out;
    out.coord = coord;
    if (const auto* c = dynamic_cast<const Constant*>(&f)) {
        out.kind = MH_FN_CONSTANT;
        out.a = c->getValue();
        out.coord.clear();
    } else if (const auto* l = dynamic_cast<const LinearFunction*>(&f)) {
        out.kind = MH_FN_LINEAR;
        out.a = l->getSlope();
        out.b = l->getIntercept();
    } else if (const auto* s = dynamic_cast<const SimmSpline*>(&f)) {
        out.kind = MH_FN_SIMMSPLINE;
        const int n = s->getSize();
        for (int i = 0; i < n; ++i) {
            out.x.push_back(s->getX()[i]);
            out.y.push_back(s->getY()[i]);
        }
    } else if (const auto* m = dynamic_cast<const MultiplierFunction*>(&f)) {
        out = toFunction(m->getFunction(), coord);
        out.scale *= m->getScale();
    } else {
        OPENSIM_THROW(Exception, "MocoHipSolver: function type '{}' is not supported "
                                 "(Constant, LinearFunction, SimmSpline, MultiplierFunction)",
                f.getConcreteClassName());
    }
    return out;
}

// A data table as the piecewise polynomial the device evaluates: the
// GCVSplineSet the reference builds over it (GCVSplineSet(table, labels,
// degree), the splines of ExternalForce, MocoStateTrackingGoal and
// PositionMotion) converted exactly -- on [t_s, t_{s+1}] a degree-d spline
// is its Taylor polynomial at t_s, coefficient k = f^(k)(t_s) / k!.
mhb::Table toTable(const std::string& name, const TimeSeriesTable& table, int degree,
        const std::vector<std::string>& renamed = {}) {
    const auto labels = table.getColumnLabels();
    GCVSplineSet splines(table, labels, degree);
    const auto& time = table.getIndependentColumn();
    mhb::Table out;
    out.name = name;
    out.degree = degree;
    out.columns = renamed.empty() ? labels : renamed;
    out.breaks.assign(time.begin(), time.end());
    const int nseg = (int)time.size() - 1;
    const int ncol = (int)labels.size();
    out.coefs.assign((size_t)nseg * ncol * (degree + 1), 0.0);
    for (int s = 0; s < nseg; ++s) {
        const SimTK::Vector t(1, time[s]);
        for (int c = 0; c < ncol; ++c) {
            const auto& sp = *splines.getGCVSpline(c);
            double fact = 1.0;
            for (int k = 0; k <= degree; ++k) {
                if (k > 0) fact *= k;
                const double v = k == 0 ? sp.calcValue(t)
                                        : sp.calcDerivative(std::vector<int>(k, 0), t);
                out.coefs[((size_t)s * ncol + c) * (degree + 1) + k] = v / fact;
            }
        }
    }
    return out;
}

// ---- frames ----------------------------------------------------------------
// A joint frame: the body it is attached to and its offset (translation,
// body-fixed XYZ orientation), identity for a body / ground frame itself.
void frameOf(const PhysicalFrame& f, std::string& body, double loc[3], double orient[3]) {
    for (int i = 0; i < 3; ++i) loc[i] = orient[i] = 0.0;
    if (const auto* o = dynamic_cast<const PhysicalOffsetFrame*>(&f)) {
        body = o->getParentFrame().findBaseFrame().getName();
        for (int i = 0; i < 3; ++i) {
            loc[i] = o->get_translation()[i];
            orient[i] = o->get_orientation()[i];
        }
    } else {
        body = f.findBaseFrame().getName();
    }
}

mhb::Coordinate toCoordinate(const Coordinate& c) {
    mhb::Coordinate out;
    out.name = c.getName();
    out.range[0] = c.getRangeMin();
    out.range[1] = c.getRangeMax();
    out.motion_type = c.getMotionType() == Coordinate::Translational ? "translational" : "rotational";
    out.default_value = c.getDefaultValue();
    out.path = c.getAbsolutePathString();
    return out;
}

// Joint -> axes (osim.py _axes_for): Pin = rotation about the child frame's
// z, Slider = translation along x, Weld = none, CustomJoint = its
// SpatialTransform's rotations then translations.
mhb::Joint toJoint(const Joint& j) {
    mhb::Joint out;
    out.name = j.getName();
    frameOf(j.getParentFrame(), out.parent, out.loc_in_parent, out.orient_in_parent);
    std::string child;
    frameOf(j.getChildFrame(), child, out.loc_in_child, out.orient_in_child);
    out.child = child;
    for (int i = 0; i < j.numCoordinates(); ++i) out.coordinates.push_back(toCoordinate(j.get_coordinates(i)));
    auto linear = [](const std::string& coord) {
        mhb::Function f;
        f.kind = MH_FN_LINEAR;
        f.coord = coord;
        f.a = 1.0;
        return f;
    };
    if (dynamic_cast<const PinJoint*>(&j)) {
        mhb::Axis a;
        a.type = MH_AXIS_ROTATION;
        a.func = linear(out.coordinates.at(0).name);
        out.axes.push_back(a);
    } else if (dynamic_cast<const SliderJoint*>(&j)) {
        mhb::Axis a;
        a.type = MH_AXIS_TRANSLATION;
        a.dir[0] = 1; a.dir[1] = 0; a.dir[2] = 0;
        a.func = linear(out.coordinates.at(0).name);
        out.axes.push_back(a);
    } else if (dynamic_cast<const WeldJoint*>(&j)) {
        // no axes
    } else if (const auto* cj = dynamic_cast<const CustomJoint*>(&j)) {
        const SpatialTransform& st = cj->getSpatialTransform();
        for (int i = 0; i < 6; ++i) {
            const TransformAxis& ta = st.getTransformAxis(i);
            const auto names = ta.getCoordinateNames();
            OPENSIM_THROW_IF(names.size() > 1, Exception,
                    "MocoHipSolver: TransformAxis of joint '{}' with more than one coordinate", j.getName());
            const std::string coord = names.size() ? names[0] : std::string();
            mhb::Axis a;
            a.type = i < 3 ? MH_AXIS_ROTATION : MH_AXIS_TRANSLATION;
            for (int d = 0; d < 3; ++d) a.dir[d] = ta.getAxis()[d];
            a.func = ta.hasFunction() ? toFunction(ta.getFunction(), coord) : mhb::Function{};
            OPENSIM_THROW_IF(coord.empty() && a.func.kind != MH_FN_CONSTANT, Exception,
                    "MocoHipSolver: non-constant TransformAxis without a coordinate in '{}'", j.getName());
            out.axes.push_back(a);
        }
    } else {
        OPENSIM_THROW(Exception, "MocoHipSolver: joint type '{}' is not supported",
                j.getConcreteClassName());
    }
    return out;
}

// ---- muscles and paths -------------------------------------------------------
mhb::Muscle toMuscle(const DeGrooteFregly2016Muscle& m) {
    mhb::Muscle out;
    out.name = m.getName();
    out.path = m.getAbsolutePathString();
    out.max_isometric_force = m.get_max_isometric_force();
    out.optimal_fiber_length = m.get_optimal_fiber_length();
    out.tendon_slack_length = m.get_tendon_slack_length();
    out.pennation_angle_at_optimal = m.get_pennation_angle_at_optimal();
    out.max_contraction_velocity = m.get_max_contraction_velocity();
    out.activation_time_constant = m.get_activation_time_constant();
    out.deactivation_time_constant = m.get_deactivation_time_constant();
    out.default_activation = m.get_default_activation();
    out.default_normalized_tendon_force = m.get_default_normalized_tendon_force();
    out.active_force_width_scale = m.get_active_force_width_scale();
    out.fiber_damping = m.get_fiber_damping();
    out.passive_fiber_strain_at_one_norm_force = m.get_passive_fiber_strain_at_one_norm_force();
    out.tendon_strain_at_one_norm_force = m.get_tendon_strain_at_one_norm_force();
    out.ignore_passive_fiber_force = m.get_ignore_passive_fiber_force();
    out.ignore_activation_dynamics = m.get_ignore_activation_dynamics();
    out.ignore_tendon_compliance = m.get_ignore_tendon_compliance();
    out.tendon_compliance_dynamics_mode = m.get_tendon_compliance_dynamics_mode();
    out.min_control = m.getMinControl();
    out.max_control = m.getMaxControl();
    const GeometryPath& gp = m.getGeometryPath();
    const PathPointSet& pps = gp.getPathPointSet();
    for (int i = 0; i < pps.getSize(); ++i) {
        const AbstractPathPoint& ap = pps.get(i);
        mhb::PathPoint p;
        p.name = ap.getName();
        p.body = ap.getParentFrame().findBaseFrame().getName();
        if (const auto* mp = dynamic_cast<const MovingPathPoint*>(&ap)) {
            p.kind = MH_PP_MOVING;
            if (mp->hasXLocation()) p.fx = toFunction(mp->get_x_location(), mp->getXCoordinate().getName());
            if (mp->hasYLocation()) p.fy = toFunction(mp->get_y_location(), mp->getYCoordinate().getName());
            if (mp->hasZLocation()) p.fz = toFunction(mp->get_z_location(), mp->getZCoordinate().getName());
        } else if (const auto* cp = dynamic_cast<const ConditionalPathPoint*>(&ap)) {
            p.kind = MH_PP_CONDITIONAL;
            for (int d = 0; d < 3; ++d) p.loc[d] = cp->get_location()[d];
            p.coord = cp->getCoordinate().getName();
            p.range[0] = cp->get_range(0);
            p.range[1] = cp->get_range(1);
        } else if (const auto* fp = dynamic_cast<const PathPoint*>(&ap)) {
            p.kind = MH_PP_FIXED;
            for (int d = 0; d < 3; ++d) p.loc[d] = fp->get_location()[d];
        } else {
            OPENSIM_THROW(Exception, "MocoHipSolver: path point type '{}' of '{}' is not supported",
                    ap.getConcreteClassName(), m.getName());
        }
        out.points.push_back(p);
    }
    // PathWrapSet (the muscles DeGrooteFregly2016Muscle::replaceMuscles
    // creates carry none: it copies the PathPointSet only,
    // DeGrooteFregly2016Muscle.cpp:1007-1020)
    const PathWrapSet& ws = gp.getWrapSet();
    for (int i = 0; i < ws.getSize(); ++i) {
        const PathWrap& w = ws.get(i);
        mhb::PathWrapRef r;
        r.wrap = w.getWrapObjectName();
        r.range_begin = w.getStartPoint();
        r.range_end = w.getEndPoint();
        out.path_wraps.push_back(r);
    }
    return out;
}

// ---- the model ---------------------------------------------------------------
void compileModel(const Model& model, mhb::Problem& prob) {
    mhb::Model& m = prob.model;
    m.name = model.getName();
    const SimTK::Vec3 g = model.getGravity();
    for (int i = 0; i < 3; ++i) m.gravity[i] = g[i];
    for (const Body& b : model.getComponentList<Body>()) {
        mhb::Body hb;
        hb.name = b.getName();
        hb.mass = b.getMass();
        for (int i = 0; i < 3; ++i) hb.com[i] = b.getMassCenter()[i];
        const SimTK::Inertia I = b.getInertia();
        for (int i = 0; i < 3; ++i) {
            hb.inertia[i] = I.getMoments()[i];
            hb.inertia[3 + i] = I.getProducts()[i];
        }
        m.add_body(hb);
        for (const WrapObject& w : b.getComponentList<WrapObject>()) {
            const auto* wc = dynamic_cast<const WrapCylinder*>(&w);
            OPENSIM_THROW_IF(!wc, Exception, "MocoHipSolver: wrap object '{}' ({}) is not a WrapCylinder",
                    w.getName(), w.getConcreteClassName());
            mhb::WrapCylinder hw;
            hw.name = wc->getName();
            hw.body = b.getName();
            hw.radius = wc->get_radius();
            hw.length = wc->get_length();
            for (int d = 0; d < 3; ++d) {
                hw.xyz_body_rotation[d] = wc->get_xyz_body_rotation()[d];
                hw.translation[d] = wc->get_translation()[d];
            }
            hw.quadrant = wc->get_quadrant();
            hw.active = wc->get_active();
            m.add_wrap(hw);
        }
    }
    for (const Joint& j : model.getComponentList<Joint>()) m.add_joint(toJoint(j));
    // actuators in force-set order (MocoUtilities.cpp:557-587)
    for (const Actuator& a : model.getComponentList<Actuator>()) {
        if (!a.get_appliesForce()) continue;
        if (const auto* mu = dynamic_cast<const DeGrooteFregly2016Muscle*>(&a)) {
            m.add_muscle(toMuscle(*mu));
        } else if (const auto* ca = dynamic_cast<const CoordinateActuator*>(&a)) {
            mhb::CoordinateActuator hc;
            hc.name = ca->getName();
            hc.path = ca->getAbsolutePathString();
            hc.coordinate = ca->getCoordinate()->getName();
            hc.optimal_force = ca->getOptimalForce();
            hc.min_control = ca->getMinControl();
            hc.max_control = ca->getMaxControl();
            m.add_coordinate_actuator(hc);
        } else {
            OPENSIM_THROW(Exception, "MocoHipSolver: actuator '{}' of type '{}' is not supported "
                                     "(DeGrooteFregly2016Muscle, CoordinateActuator)",
                    a.getName(), a.getConcreteClassName());
        }
    }
    // SpringGeneralizedForces (-stiffness (q - rest_length) - viscosity u on
    // their coordinate; testMocoParameters.cpp:50-55)
    for (const SpringGeneralizedForce& f : model.getComponentList<SpringGeneralizedForce>()) {
        if (!f.get_appliesForce()) continue;
        mhb::SpringGeneralizedForce hs;
        hs.name = f.getName();
        hs.path = f.getAbsolutePathString();
        hs.coordinate = f.get_coordinate();
        hs.stiffness = f.getStiffness();
        hs.rest_length = f.getRestLength();
        hs.viscosity = f.getViscosity();
        m.add_spring(hs);
    }
    // ExternalForces on ground-expressed data (ModOpAddExternalLoads): one
    // table per data source, cubic GCV splines as ExternalForce builds them
    int ntab = 0;
    for (const ExternalForce& ef : model.getComponentList<ExternalForce>()) {
        OPENSIM_THROW_IF(ef.get_force_expressed_in_body() != "ground" || ef.get_point_expressed_in_body() != "ground",
                Exception, "MocoHipSolver: ExternalForce '{}' must be expressed in ground", ef.getName());
        const Storage& data = ef.getDataSource();
        TimeSeriesTable tt = data.exportToTable();
        const std::string tname = "grf" + std::to_string(ntab++);
        m.add_table(toTable(tname, tt, 3));
        mhb::ExternalForce he;
        he.name = ef.getName();
        he.body = ef.get_applied_to_body();
        he.table = tname;
        he.force_identifier = ef.get_force_identifier();
        he.point_identifier = ef.get_point_identifier();
        he.torque_identifier = ef.get_torque_identifier();
        m.add_external_force(he);
    }
    for (const Marker& mk : model.getComponentList<Marker>()) {
        mhb::Marker hm;
        hm.name = mk.getName();
        hm.path = mk.getAbsolutePathString();
        hm.body = mk.getParentFrame().findBaseFrame().getName();
        for (int d = 0; d < 3; ++d) hm.location[d] = mk.get_location()[d];
        m.add_marker(hm);
    }
    for (const CoordinateCouplerConstraint& k : model.getComponentList<CoordinateCouplerConstraint>()) {
        if (!k.isEnforced(model.getWorkingState())) continue;
        const auto ind = k.getIndependentCoordinateNames();
        OPENSIM_THROW_IF(ind.size() != 1, Exception,
                "MocoHipSolver: CoordinateCouplerConstraint '{}' with {} independent coordinates",
                k.getName(), ind.size());
        mhb::CoordinateCoupler hk;
        hk.name = k.getName();
        hk.dependent = k.getDependentCoordinateName();
        hk.function = toFunction(k.getFunction(), ind[0]);
        hk.scale_factor = k.get_scale_factor();
        m.add_constraint(hk);
    }
}

mhb::Bounds toBounds(const MocoBounds& b) {
    mhb::Bounds out;
    if (b.isSet()) {
        out.lower = b.getLower();
        out.upper = b.getUpper();
    }
    return out;
}

mhb::BoundFunction toBoundFunction(const Function& f) {
    mhb::BoundFunction out;
    if (const auto* c = dynamic_cast<const Constant*>(&f)) {
        out.kind = mhb::BoundFunction::CONSTANT;
        out.value = c->getValue();
    } else if (const auto* p = dynamic_cast<const PiecewiseLinearFunction*>(&f)) {
        out.kind = mhb::BoundFunction::PIECEWISE_LINEAR;
        for (int i = 0; i < p->getSize(); ++i) {
            out.x.push_back(p->getX(i));
            out.y.push_back(p->getY(i));
        }
    } else if (const auto* s = dynamic_cast<const GCVSpline*>(&f)) {
        // the spline over its own knots as a piecewise polynomial (toTable)
        TimeSeriesTable t;
        t.setColumnLabels({"bound"});
        for (int i = 0; i < s->getSize(); ++i) t.appendRow(s->getX()[i], SimTK::RowVector(1, s->getY()[i]));
        const mhb::Table tb = toTable("bound", t, s->getDegree());
        out.kind = mhb::BoundFunction::SPLINE;
        out.x = tb.breaks;
        out.breaks = tb.breaks;
        out.coefs = tb.coefs;
        out.degree = tb.degree;
    } else {
        OPENSIM_THROW(Exception, "MocoHipSolver: bound function '{}' is not supported", f.getConcreteClassName());
    }
    return out;
}

}  // namespace

// ---- compileProblemRep --------------------------------------------------------
mhb::Problem OpenSim::compileProblemRep(const MocoProblemRep& rep) {
    mhb::Problem prob;
    const Model& model = rep.getModelBase();
    compileModel(model, prob);
    prob.time_initial = toBounds(rep.getTimeInitialBounds());
    prob.time_final = toBounds(rep.getTimeFinalBounds());
    for (const std::string& n : rep.createStateInfoNames()) {
        const MocoVariableInfo& vi = rep.getStateInfo(n);
        prob.state_infos.push_back({n, {toBounds(vi.getBounds()), toBounds(vi.getInitialBounds()),
                                        toBounds(vi.getFinalBounds())}});
    }
    for (const std::string& n : rep.createControlInfoNames()) {
        const MocoVariableInfo& vi = rep.getControlInfo(n);
        prob.control_infos.push_back({n, {toBounds(vi.getBounds()), toBounds(vi.getInitialBounds()),
                                          toBounds(vi.getFinalBounds())}});
    }
    // prescribed kinematics (MocoInverse's PositionMotion, MocoInverse.cpp:
    // 46-66): its coordinate functions as one table, columns = value paths
    if (rep.isPrescribedKinematics()) {
        const auto& pm = model.getComponentList<PositionMotion>().begin();
        TimeSeriesTable samples;
        std::vector<std::string> cols;
        const auto coords = model.getCoordinatesInMultibodyTreeOrder();
        // sample each coordinate's function at its own knots (GCVSplines of
        // a common time column, PositionMotion::createFromTable)
        const FunctionSet& fs = pm->get_functions();
        const auto* first = dynamic_cast<const GCVSpline*>(&fs.get(0));
        OPENSIM_THROW_IF(!first, Exception, "MocoHipSolver: PositionMotion functions must be GCVSplines");
        std::vector<std::string> labels;
        for (int i = 0; i < fs.getSize(); ++i) labels.push_back(fs.get(i).getName());
        samples.setColumnLabels(labels);
        for (int r = 0; r < first->getSize(); ++r) {
            SimTK::RowVector row(fs.getSize());
            for (int i = 0; i < fs.getSize(); ++i) row[i] = dynamic_cast<const GCVSpline&>(fs.get(i)).getY()[r];
            samples.appendRow(first->getX()[r], row);
        }
        prob.position_motion = toTable("kinematics", samples, first->getDegree());
    }
    // goals: costs, then the endpoint constraints (MocoProblemRep::
    // createEndpointConstraintNames order)
    auto addGoal = [&](const MocoGoal& g) {
        mhb::Goal hg;
        hg.name = g.getName();
        hg.weight = g.getWeight();
        if (const auto* c = dynamic_cast<const MocoControlGoal*>(&g)) {
            hg.kind = mhb::Goal::CONTROL;
            hg.exponent = c->getExponent();
            const MocoWeightSet& ws = c->get_control_weights();
            for (int i = 0; i < ws.getSize(); ++i) hg.weights.push_back({ws.get(i).getName(), ws.get(i).getWeight()});
        } else if (const auto* s = dynamic_cast<const MocoStateTrackingGoal*>(&g)) {
            hg.kind = mhb::Goal::STATE_TRACKING;
            TimeSeriesTable ref = s->getReference().process(&model);
            hg.table = "state_reference_" + g.getName();
            prob.model.add_table(toTable(hg.table, ref, 5));
            const MocoWeightSet& ws = s->get_states_weight_set();
            for (int i = 0; i < ws.getSize(); ++i) hg.weights.push_back({ws.get(i).getName(), ws.get(i).getWeight()});
        } else if (dynamic_cast<const MocoFinalTimeGoal*>(&g)) {
            hg.kind = mhb::Goal::FINAL_TIME;
        } else if (const auto* q = dynamic_cast<const MocoSumSquaredStateGoal*>(&g)) {
            hg.kind = mhb::Goal::SUM_SQUARED_STATE;
            const MocoWeightSet& ws = q->get_state_weights();
            for (int i = 0; i < ws.getSize(); ++i) hg.weights.push_back({ws.get(i).getName(), ws.get(i).getWeight()});
        } else if (dynamic_cast<const MocoInitialActivationGoal*>(&g)) {
            hg.kind = mhb::Goal::INITIAL_ACTIVATION;
            hg.mode = g.getModeAsString() == "cost" ? "cost" : "endpoint_constraint";
        } else if (const auto* mf = dynamic_cast<const MocoMarkerFinalGoal*>(&g)) {
            hg.kind = mhb::Goal::MARKER_FINAL;
            hg.point_name = mf->get_point_name();
            for (int d = 0; d < 3; ++d) hg.reference_location[d] = mf->get_reference_location()[d];
        } else {
            OPENSIM_THROW(Exception, "MocoHipSolver: goal '{}' of type '{}' is not supported (SURVEY §8 A11)",
                    g.getName(), g.getConcreteClassName());
        }
        prob.goals.push_back(hg);
    };
    for (int i = 0; i < rep.getNumCosts(); ++i) addGoal(rep.getCostByIndex(i));
    for (int i = 0; i < rep.getNumEndpointConstraints(); ++i) addGoal(rep.getEndpointConstraintByIndex(i));
    // path constraints (MocoControlBoundConstraint only)
    for (int i = 0; i < rep.getNumPathConstraints(); ++i) {
        const MocoPathConstraint& pc = rep.getPathConstraintByIndex(i);
        const auto* cb = dynamic_cast<const MocoControlBoundConstraint*>(&pc);
        OPENSIM_THROW_IF(!cb, Exception, "MocoHipSolver: path constraint '{}' of type '{}' is not supported",
                pc.getName(), pc.getConcreteClassName());
        mhb::ControlBoundConstraint hc;
        hc.name = cb->getName();
        for (const auto& p : cb->getControlPaths()) hc.control_paths.push_back(p);
        if (cb->hasLowerBound()) hc.lower = toBoundFunction(cb->getLowerBound());
        if (cb->hasUpperBound()) hc.upper = toBoundFunction(cb->getUpperBound());
        hc.equality_with_lower = cb->getEqualityWithLower();
        prob.path_constraints.push_back(hc);
    }
    // MocoParameters in createParameterNames order (the x layout's last
    // block); mhb::make_rep resolves the component paths and properties and
    // throws MocoParameter::initializeOnModel's errors for the rest (a
    // property this build does not parameterize, e.g. optimal_fiber_length,
    // is refused there by name)
    for (const std::string& name : rep.createParameterNames()) {
        const MocoParameter& par = rep.getParameter(name);
        mhb::Parameter hp;
        hp.name = name;
        hp.component_paths = par.getComponentPaths();
        hp.property_name = par.getPropertyName();
        hp.bounds = toBounds(par.getBounds());
        hp.property_element = par.getProperty_property_element().size() ? par.get_property_element() : -1;
        prob.parameters.push_back(hp);
    }
    return prob;
}

// ---- the solver ----------------------------------------------------------------
MocoHipSolver::MocoHipSolver() { constructProperties(); }

void MocoHipSolver::constructProperties() {
    constructProperty_optim_finite_difference_scheme("central");
    constructProperty_optim_sparsity_detection("none");
    constructProperty_device(0);
    constructProperty_jacobian_mode("callback-fd");
}

mhb::SolverSettings MocoHipSolver::settings() const {
    mhb::SolverSettings s;
    s.num_mesh_intervals = get_num_mesh_intervals();
    s.transcription_scheme = get_transcription_scheme();
    s.interpolate_control_midpoints = get_interpolate_control_midpoints();
    s.optim_finite_difference_scheme = get_optim_finite_difference_scheme();
    s.device = get_device();
    s.multibody_dynamics_mode = get_multibody_dynamics_mode();
    s.implicit_multibody_acceleration_bounds[0] = get_implicit_multibody_acceleration_bounds().getLower();
    s.implicit_multibody_acceleration_bounds[1] = get_implicit_multibody_acceleration_bounds().getUpper();
    s.implicit_auxiliary_derivative_bounds[0] = get_implicit_auxiliary_derivative_bounds().getLower();
    s.implicit_auxiliary_derivative_bounds[1] = get_implicit_auxiliary_derivative_bounds().getUpper();
    s.enforce_constraint_derivatives = get_enforce_constraint_derivatives();
    s.minimize_lagrange_multipliers = get_minimize_lagrange_multipliers();
    s.lagrange_multiplier_weight = get_lagrange_multiplier_weight();
    s.velocity_correction_bounds[0] = get_velocity_correction_bounds().getLower();
    s.velocity_correction_bounds[1] = get_velocity_correction_bounds().getUpper();
    s.jacobian_mode = get_jacobian_mode();
    s.optim_sparsity_detection = get_optim_sparsity_detection();
    s.optim_sparsity_detection_random_count = 3;   // MocoCasADiSolver.cpp:251
    return s;
}

void MocoHipSolver::setGuess(MocoTrajectory guess) {
    clearGuess();
    m_guessFromAPI = std::move(guess);
}
void MocoHipSolver::setGuessFile(const std::string& file) {
    clearGuess();
    set_guess_file(file);
}
void MocoHipSolver::clearGuess() {
    m_guessFromAPI = MocoTrajectory();
    m_guessFromFile = MocoTrajectory();
    set_guess_file("");
    m_guessToUse.reset();
}
const MocoTrajectory& MocoHipSolver::getGuess() const {
    if (!m_guessToUse) {
        if (get_guess_file() != "" && m_guessFromFile.getRef().empty()) {
            m_guessFromFile = MocoTrajectory(get_guess_file());
            m_guessToUse.reset(&m_guessFromFile.getRef());
        } else if (!m_guessFromAPI.empty()) {
            m_guessToUse.reset(&m_guessFromAPI);
        } else {
            m_guessToUse.reset(&m_guessFromFile.getRef());   // empty: the bounds guess
        }
    }
    return m_guessToUse.getRef();
}

namespace {

// The trajectory conversions of the reference (MocoCasOCProblem.h:70-187:
// convertToCasOCIterate / convertToMocoTrajectory) over every variable block
// by name -- states, controls, multipliers, derivatives, slacks -- shared
// with the command-line path (csrc/host/mh_trajectory.hpp; mh_build
// --solution writes the same MocoSolution as a .sto, tests/
// test_trajectory_cpp.py checks it against the Python conversion and the
// reference's MocoInverse solution file).
mhb::TrajectoryTable toTable(const MocoTrajectory& t) {
    mhb::TrajectoryTable T;
    const SimTK::Vector time = t.getTime();
    for (int k = 0; k < time.size(); ++k) T.time.push_back(time[k]);
    auto take = [&](const std::vector<std::string>& names, const SimTK::Matrix& M, std::vector<std::string>& tn,
                    std::vector<double>& td) {
        tn = names;
        td.assign((size_t)M.nrow() * M.ncol(), 0.0);
        for (int k = 0; k < M.nrow(); ++k)
            for (int j = 0; j < M.ncol(); ++j) td[(size_t)k * M.ncol() + j] = M(k, j);
    };
    take(t.getStateNames(), t.getStatesTrajectory(), T.state_names, T.states);
    take(t.getControlNames(), t.getControlsTrajectory(), T.control_names, T.controls);
    take(t.getMultiplierNames(), t.getMultipliersTrajectory(), T.multiplier_names, T.multipliers);
    take(t.getDerivativeNames(), t.getDerivativesTrajectory(), T.derivative_names, T.derivatives);
    take(t.getSlackNames(), t.getSlacksTrajectory(), T.slack_names, T.slacks);
    T.parameter_names = t.getParameterNames();
    const SimTK::RowVector& pv = t.getParameters();
    for (int j = 0; j < pv.size(); ++j) T.parameters.push_back(pv[j]);
    return T;
}

// The guess resampled at the grid times (CasOCTranscription.cpp:593-597),
// then every block it names into the iterate; unnamed blocks stay 0.
std::vector<double> toIterate(MocoTrajectory guess, const mhb::ProblemRep& hrep, const mh_options& o) {
    const auto t = guess.getTime();
    const auto times = mhb::grid_times(o, t[0], t[t.size() - 1]);
    guess.resample(SimTK::Vector((int)times.size(), times.data()));
    return mhb::trajectory_to_iterate(toTable(guess), hrep, o);
}

// The solution iterate as a MocoSolution at the grid times, every block by
// name; the slacks appended the reference's way (convertToMocoTrajectory:
// the N interval values placed uniformly over [t0, tf] and interpolated
// onto the grid).
MocoSolution toSolution(const std::vector<double>& x, const mhb::ProblemRep& hrep, const mh_options& o) {
    const mhb::TrajectoryTable T = mhb::iterate_to_trajectory(x, hrep, o);
    const int G = (int)T.time.size();
    auto matrix = [&](const std::vector<double>& d, size_t nv) {
        SimTK::Matrix M(G, (int)nv);
        for (int k = 0; k < G; ++k)
            for (size_t j = 0; j < nv; ++j) M(k, (int)j) = d[(size_t)k * nv + j];
        return M;
    };
    SimTK::RowVector parameters((int)T.parameters.size());
    for (int j = 0; j < parameters.size(); ++j) parameters[j] = T.parameters[(size_t)j];
    MocoSolution sol(SimTK::Vector(G, T.time.data()), T.state_names, T.control_names, T.multiplier_names,
            T.derivative_names, T.parameter_names, matrix(T.states, T.state_names.size()),
            matrix(T.controls, T.control_names.size()), matrix(T.multipliers, T.multiplier_names.size()),
            matrix(T.derivatives, T.derivative_names.size()), parameters);
    const int N = o.num_mesh_intervals;
    const int nsl = (int)T.slack_names.size();
    if (nsl) {
        const SimTK::Vector slackTime = createVectorLinspace(N, T.time.front(), T.time.back());
        for (int l = 0; l < nsl; ++l) {
            SimTK::Vector v(N);
            for (int i = 0; i < N; ++i) v[i] = T.slacks[(size_t)(2 * i + 1) * nsl + l];   // the midpoints
            sol.appendSlack(T.slack_names[l], interpolate(slackTime, v, sol.getTime()));
        }
    }
    return sol;
}

// Ipopt's return status by name (IpReturnCodes_inc.h), as MocoCasADiSolver
// reports CasADi's "return_status".
std::string ipoptStatusName(Ipopt::ApplicationReturnStatus s) {
    switch (s) {
    case Ipopt::Solve_Succeeded: return "Solve_Succeeded";
    case Ipopt::Solved_To_Acceptable_Level: return "Solved_To_Acceptable_Level";
    case Ipopt::Infeasible_Problem_Detected: return "Infeasible_Problem_Detected";
    case Ipopt::Search_Direction_Becomes_Too_Small: return "Search_Direction_Becomes_Too_Small";
    case Ipopt::Diverging_Iterates: return "Diverging_Iterates";
    case Ipopt::User_Requested_Stop: return "User_Requested_Stop";
    case Ipopt::Feasible_Point_Found: return "Feasible_Point_Found";
    case Ipopt::Maximum_Iterations_Exceeded: return "Maximum_Iterations_Exceeded";
    case Ipopt::Restoration_Failed: return "Restoration_Failed";
    case Ipopt::Error_In_Step_Computation: return "Error_In_Step_Computation";
    case Ipopt::Maximum_CpuTime_Exceeded: return "Maximum_CpuTime_Exceeded";
    case Ipopt::Not_Enough_Degrees_Of_Freedom: return "Not_Enough_Degrees_Of_Freedom";
    case Ipopt::Invalid_Problem_Definition: return "Invalid_Problem_Definition";
    case Ipopt::Invalid_Option: return "Invalid_Option";
    case Ipopt::Invalid_Number_Detected: return "Invalid_Number_Detected";
    default: return "Ipopt status " + std::to_string((int)s);
    }
}

// The context owned for the solve: destroyed on every exit path.
struct CtxGuard {
    mh_ctx* ctx = nullptr;
    ~CtxGuard() { mh_destroy(ctx); }
};

}  // namespace

MocoSolution MocoHipSolver::solveImpl() const {
    const Stopwatch stopwatch;
    const MocoProblemRep& rep = getProblemRep();
    if (get_verbosity()) {
        log_info(std::string(72, '='));
        log_info("MocoHipSolver starting (MI355X direct-collocation hot path).");
        rep.printDescription();
    }
    // lower the problem and transcribe it on the device
    const mhb::Problem prob = compileProblemRep(rep);
    mhb::ProblemRep hrep;
    mhb::make_rep(prob, hrep);
    mh_options opt = mhb::make_options(settings());
    // the starting point: the user's guess resampled on the grid, every
    // block by name, else the bounds-midpoint guess (MocoCasADiSolver.cpp:
    // 326-332); "initial-guess" sparsity detection probes at it
    // (CasOCSolver.cpp:74-76; null: the bounds midpoint, the same guess)
    std::vector<double> x0;
    const MocoTrajectory& guess = getGuess();
    if (!guess.empty()) x0 = toIterate(guess, hrep, opt);
    // the library's n before mh_create reads the guess (n doubles): the
    // host-only layout query, so a layout mismatch is an error, not a read
    // past the iterate
    mh_nlp_info layout{};
    OPENSIM_THROW_IF(mh_get_nlp_info_for(&hrep.problem, &opt, &layout) != MH_OK, Exception,
            "MocoHipSolver: {}", mh_last_error());
    OPENSIM_THROW_IF(!x0.empty() && (int64_t)x0.size() != layout.n, Exception,
            "MocoHipSolver: the guess iterate has {} values, the problem has n = {}", x0.size(), layout.n);
    if (opt.sparsity_detection == MH_SPARSITY_INITIAL_GUESS) opt.sparsity_guess = x0.empty() ? nullptr : x0.data();
    CtxGuard ctx;
    OPENSIM_THROW_IF(mh_create(&hrep.problem, &opt, &ctx.ctx) != MH_OK, Exception,
            "MocoHipSolver: mh_create failed: {}", mh_last_error());
    Ipopt::SmartPtr<mocohip::MocoHipTNLP> tnlp = new mocohip::MocoHipTNLP(ctx.ctx, x0);
    mocohip::IpoptSettings ips;
    ips.verbosity = get_verbosity();
    ips.optim_max_iterations = get_optim_max_iterations();
    ips.optim_convergence_tolerance = get_optim_convergence_tolerance();
    ips.optim_constraint_tolerance = get_optim_constraint_tolerance();
    ips.optim_hessian_approximation = get_optim_hessian_approximation();
    ips.optim_ipopt_print_level = get_optim_ipopt_print_level();
    const Ipopt::ApplicationReturnStatus status = mocohip::solve(tnlp, ips);
    MocoSolution solution = toSolution(tnlp->solution(), hrep, opt);
    // the objective's terms at the solution, one per cost goal
    // (MocoCasADiSolver.cpp:395-402: the solution's objective breakdown)
    std::vector<std::pair<std::string, double>> breakdown;
    const std::vector<std::string> costs = rep.createCostNames();
    std::vector<double> terms(costs.size() + 1, 0.0);
    int32_t nterms = (int32_t)terms.size();
    if (mh_eval_objective_terms(ctx.ctx, tnlp->solution().data(), terms.data(), &nterms) == MH_OK)
        for (int i = 0; i < (int)costs.size() && i < nterms; ++i) breakdown.emplace_back(costs[i], terms[i]);
    const long long elapsed = stopwatch.getElapsedTimeInNs();
    const bool success = status == Ipopt::Solve_Succeeded || status == Ipopt::Solved_To_Acceptable_Level;
    setSolutionStats(solution, success, tnlp->objective(), ipoptStatusName(status), tnlp->iterations(),
            SimTK::nsToSec(elapsed), breakdown);
    if (get_verbosity()) {
        log_info("Elapsed real time: {}.", stopwatch.formatNs(elapsed));
        log_info(std::string(72, '='));
    }
    return solution;
}
