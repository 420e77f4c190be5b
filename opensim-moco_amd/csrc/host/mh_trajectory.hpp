// mh_trajectory.hpp — an NLP iterate <-> a MocoTrajectory's named blocks, on
// the transcription grid, for C++ hosts over the C ABI (the MocoHipSolver
// plugin's toIterate / toSolution, integration/MocoHipSolver.cpp; mh_build
// --solution).  Header-only; no OpenSim, no GPU.
//
// The reference converts in both directions with every variable block by
// name -- states, controls, multipliers, slacks, derivatives, parameters
// (MocoCasOCProblem.h:70-100 convertToCasOCIterate, :128-187
// convertToMocoTrajectory) -- over CasOC's x layout (CasOCIterate.h:27-44,
// include/mocohip.h): t0, tf, states NS x G grid-major, controls NC x G,
// multipliers NM x G, slacks NSL x N (one per mesh interval, at the
// Hermite-Simpson midpoints), derivatives NDV x G (accelerations of implicit
// multibody dynamics, then implicit auxiliary derivatives), parameters NPAR
// (MocoParameters, CasOCIterate.h: Var::parameters).
#ifndef MOCOHIP_HOST_MH_TRAJECTORY_HPP
#define MOCOHIP_HOST_MH_TRAJECTORY_HPP

#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "mh_builder.hpp"

namespace mhb {

// The block sizes of one transcription (what mh_get_nlp_info reports,
// computed from the rep and options without a context).
struct IterateLayout {
    int N = 0, G = 0, NS = 0, NC = 0, NM = 0, NSL = 0, NACC = 0, NAR = 0, NPAR = 0;
    bool hs = true;
    int NDV() const { return NACC + NAR; }
    long n() const { return 2 + (long)(NS + NC + NM + NDV()) * G + (long)NSL * N + NPAR; }
    long off_controls() const { return 2 + (long)NS * G; }
    long off_multipliers() const { return off_controls() + (long)NC * G; }
    long off_slacks() const { return off_multipliers() + (long)NM * G; }
    long off_derivatives() const { return off_slacks() + (long)NSL * N; }
    long off_parameters() const { return off_derivatives() + (long)NDV() * G; }
};

inline IterateLayout iterate_layout(const ProblemRep& R, const mh_options& o) {
    IterateLayout L;
    L.N = o.num_mesh_intervals;
    L.hs = o.transcription == MH_HERMITE_SIMPSON;
    L.G = L.hs ? 2 * L.N + 1 : L.N + 1;
    L.NS = (int)R.state_names.size();
    L.NC = (int)R.control_names.size();
    L.NM = (int)R.multiplier_names.size();
    const bool presc = R.problem.prescribed_kinematics != 0;
    // velocity-correction slacks: Hermite-Simpson with enforced constraint
    // derivatives, not with prescribed kinematics (CasOCTranscription.cpp:
    // 234-241, CasOCProblem.h:508-521)
    L.NSL = (L.hs && !o.ignore_constraint_derivatives && !presc) ? L.NM : 0;
    L.NACC = (o.multibody_dynamics_mode == MH_DYNAMICS_IMPLICIT && !presc) ? R.cm.model.nq : 0;
    L.NAR = R.num_aux_residuals;
    L.NPAR = (int)R.parameter_bounds.size();
    return L;
}

// The grid times at (t0, tf): CasOCTranscription.h:40-43, times = (tf - t0)
// grid + t0 on the uniform mesh, Hermite-Simpson midpoints in between.
inline std::vector<double> grid_times(const mh_options& o, double t0, double tf) {
    const int N = o.num_mesh_intervals;
    const bool hs = o.transcription == MH_HERMITE_SIMPSON;
    std::vector<double> t;
    for (int k = 0; k < (hs ? 2 * N + 1 : N + 1); ++k) {
        const double g = hs ? ((k % 2 == 0) ? (k / 2) / (double)N
                                            : 0.5 * ((k / 2) / (double)N + (k / 2 + 1) / (double)N))
                            : k / (double)N;
        t.push_back((tf - t0) * g + t0);
    }
    return t;
}

// A MocoTrajectory's data on the grid: per block its names and a row-major
// [G][names] matrix (slacks: NaN away from the Hermite-Simpson midpoints,
// where the transcription holds none; parameters: one row).
struct TrajectoryTable {
    std::vector<double> time;
    std::vector<std::string> state_names, control_names, multiplier_names, derivative_names, slack_names,
            parameter_names;
    std::vector<double> states, controls, multipliers, derivatives, slacks, parameters;
};

inline std::vector<std::string> derivative_names(const ProblemRep& R, const IterateLayout& L) {
    std::vector<std::string> d;
    for (int j = 0; j < L.NACC; ++j)
        d.push_back(j < (int)R.accel_names.size() ? R.accel_names[j] : "accel_" + std::to_string(j));
    for (int j = 0; j < L.NAR; ++j)
        d.push_back(j < (int)R.aux_derivative_names.size() ? R.aux_derivative_names[j]
                                                           : "derivative_" + std::to_string(L.NACC + j));
    return d;
}

// x -> the trajectory (convertToMocoTrajectory over expandVariables).
inline TrajectoryTable iterate_to_trajectory(const std::vector<double>& x, const ProblemRep& R,
        const mh_options& o) {
    const IterateLayout L = iterate_layout(R, o);
    if ((long)x.size() != L.n()) throw std::runtime_error("iterate size does not match the problem and grid");
    TrajectoryTable T;
    T.time = grid_times(o, x[0], x[1]);
    const int G = L.G;
    T.state_names = R.state_names;
    T.control_names = R.control_names;
    T.multiplier_names = R.multiplier_names;
    T.derivative_names = derivative_names(R, L);
    T.slack_names.assign(R.slack_names.begin(), R.slack_names.begin() + L.NSL);
    T.parameter_names = R.parameter_names;
    T.parameters.assign(x.begin() + L.off_parameters(), x.begin() + L.off_parameters() + L.NPAR);
    auto block = [&](long off, int nv, std::vector<double>& out) {
        out.assign((size_t)G * nv, 0.0);
        for (int k = 0; k < G; ++k)
            for (int j = 0; j < nv; ++j) out[(size_t)k * nv + j] = x[(size_t)(off + (long)k * nv + j)];
    };
    block(2, L.NS, T.states);
    block(L.off_controls(), L.NC, T.controls);
    block(L.off_multipliers(), L.NM, T.multipliers);
    block(L.off_derivatives(), L.NDV(), T.derivatives);
    T.slacks.assign((size_t)G * L.NSL, NAN);
    for (int i = 0; i < L.N && L.NSL; ++i)
        for (int l = 0; l < L.NSL; ++l)
            T.slacks[(size_t)(2 * i + 1) * L.NSL + l] = x[(size_t)(L.off_slacks() + (long)i * L.NSL + l)];
    return T;
}

// The trajectory (already resampled onto the grid times, e.g. by OpenSim's
// MocoTrajectory::resample) -> x; blocks the guess does not name stay 0, its
// slacks are read at the midpoints (convertToCasOCIterate); parameters by
// name, a missing one at its bounds' midpoint (the bounds guess,
// CasOCTranscription.cpp:1124-1139; mocohip/trajectory.py to_iterate).
inline std::vector<double> trajectory_to_iterate(const TrajectoryTable& T, const ProblemRep& R,
        const mh_options& o) {
    const IterateLayout L = iterate_layout(R, o);
    if ((int)T.time.size() != L.G) throw std::runtime_error("the guess is not on the transcription grid");
    std::vector<double> x((size_t)L.n(), 0.0);
    x[0] = T.time.front();
    x[1] = T.time.back();
    auto fill = [&](const std::vector<std::string>& want, const std::vector<std::string>& have,
                    const std::vector<double>& data, long off, bool slacks) {
        const int nw = (int)want.size(), nh = (int)have.size();
        for (int j = 0; j < nw; ++j)
            for (int h = 0; h < nh; ++h) {
                if (have[h] != want[j]) continue;
                if (slacks) {
                    for (int i = 0; i < L.N; ++i) x[(size_t)(off + (long)i * nw + j)] = data[(size_t)(2 * i + 1) * nh + h];
                } else {
                    for (int k = 0; k < L.G; ++k) x[(size_t)(off + (long)k * nw + j)] = data[(size_t)k * nh + h];
                }
                break;
            }
    };
    fill(R.state_names, T.state_names, T.states, 2, false);
    fill(R.control_names, T.control_names, T.controls, L.off_controls(), false);
    fill(R.multiplier_names, T.multiplier_names, T.multipliers, L.off_multipliers(), false);
    fill(derivative_names(R, L), T.derivative_names, T.derivatives, L.off_derivatives(), false);
    if (L.NSL) {
        const std::vector<std::string> sn(R.slack_names.begin(), R.slack_names.begin() + L.NSL);
        fill(sn, T.slack_names, T.slacks, L.off_slacks(), true);
    }
    for (int q = 0; q < L.NPAR; ++q) {
        const mh_bounds& b = R.parameter_bounds[q];
        const bool set = !std::isnan(b.lower) && !std::isnan(b.upper);
        const double l = set ? b.lower : -INFINITY, u = set ? b.upper : INFINITY;
        double v = !std::isinf(l) && !std::isinf(u) ? 0.5 * (u + l) : !std::isinf(l) ? l : !std::isinf(u) ? u : 0.0;
        for (size_t h = 0; h < T.parameter_names.size(); ++h)
            if (T.parameter_names[h] == R.parameter_names[q] && h < T.parameters.size()) { v = T.parameters[h]; break; }
        x[(size_t)(L.off_parameters() + q)] = v;
    }
    return x;
}

// MocoTrajectory::write's .sto (MocoTrajectory.cpp: the block counts as
// header metadata, sorted, then DataType / version, endheader, a time column
// and the states, controls, multipliers, derivatives, slacks, parameters; NaN
// where a slack has no value; the parameters in the first row, NaN below,
// convertToTable).
inline void write_sto(const TrajectoryTable& T, const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) throw std::runtime_error("cannot write " + path);
    const size_t G = T.time.size();
    std::fprintf(f, "MocoHipSolution\nnum_controls=%zu\nnum_derivatives=%zu\nnum_multipliers=%zu\n"
                    "num_parameters=%zu\nnum_slacks=%zu\nnum_states=%zu\nDataType=double\nversion=3\nendheader\ntime",
                 T.control_names.size(), T.derivative_names.size(), T.multiplier_names.size(),
                 T.parameter_names.size(), T.slack_names.size(), T.state_names.size());
    for (auto* names : {&T.state_names, &T.control_names, &T.multiplier_names, &T.derivative_names,
                        &T.slack_names, &T.parameter_names})
        for (auto& n : *names) std::fprintf(f, "\t%s", n.c_str());
    std::fprintf(f, "\n");
    for (size_t k = 0; k < G; ++k) {
        std::fprintf(f, "%.17g", T.time[k]);
        auto row = [&](const std::vector<double>& d, size_t nv) {
            for (size_t j = 0; j < nv; ++j) {
                const double v = d[k * nv + j];
                if (std::isnan(v)) std::fprintf(f, "\tNaN");
                else std::fprintf(f, "\t%.17g", v);
            }
        };
        row(T.states, T.state_names.size());
        row(T.controls, T.control_names.size());
        row(T.multipliers, T.multiplier_names.size());
        row(T.derivatives, T.derivative_names.size());
        row(T.slacks, T.slack_names.size());
        for (size_t j = 0; j < T.parameter_names.size(); ++j) {
            if (k == 0 && j < T.parameters.size()) std::fprintf(f, "\t%.17g", T.parameters[j]);
            else std::fprintf(f, "\tNaN");
        }
        std::fprintf(f, "\n");
    }
    std::fclose(f);
}

}  // namespace mhb

#endif
