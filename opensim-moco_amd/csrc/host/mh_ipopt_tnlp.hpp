// Ipopt::TNLP adapter over the libmocohip C ABI.
//
// The reference's tropter IPOPTSolver::TNLP (tropter/tropter/optimization/
// IPOPTSolver.cpp:302-469) with the problem's calc_* calls replaced by mh_*
// entries: structure, bounds, starting point and values all come from the
// library, so the adapter holds no sparsity of its own.  Options follow
// MocoCasADiSolver.cpp:210-246 (the same mapping as the Python mirror
// mocohip.solver.MocoHipSolver.ipopt_options, tested in
// tests/test_trajectory.py::test_ipopt_option_mapping).
//
// NOT compiled in this repository: Ipopt 3.12.8 (IpTNLP.hpp,
// IpIpoptApplication.hpp) is not in the build image.  A
// MocoSolver plugin includes this header where Ipopt is
// installed; everything it calls on our side is exported by libmocohip.so
// and exercised by tests/ and csrc/host/mh_driver.cpp.
#pragma once

#include <IpIpoptApplication.hpp>
#include <IpIpoptData.hpp>
#include <IpTNLP.hpp>

#include <stdexcept>
#include <string>
#include <vector>

#include "mocohip.h"

namespace mocohip {

// The MocoDirectCollocationSolver / MocoCasADiSolver properties the option
// mapping reads (defaults: MocoDirectCollocationSolver.cpp:23-42).
struct IpoptSettings {
    int verbosity = 2;
    int optim_max_iterations = -1;
    double optim_convergence_tolerance = -1.0;
    double optim_constraint_tolerance = -1.0;
    std::string optim_hessian_approximation = "limited-memory";
    int optim_ipopt_print_level = -1;
};

// MocoCasADiSolver.cpp:218-246.
inline void apply_ipopt_options(Ipopt::IpoptApplication& app, const IpoptSettings& s) {
    auto opts = app.Options();
    opts->SetStringValue("print_user_options", "yes");
    if (s.verbosity < 2) opts->SetIntegerValue("print_level", 0);
    else if (s.optim_ipopt_print_level != -1) opts->SetIntegerValue("print_level", s.optim_ipopt_print_level);
    opts->SetStringValue("hessian_approximation", s.optim_hessian_approximation);
    if (s.optim_max_iterations != -1) opts->SetIntegerValue("max_iter", s.optim_max_iterations);
    if (s.optim_convergence_tolerance != -1) {
        const double tol = s.optim_convergence_tolerance;   // as Simbody does
        for (const char* k : {"tol", "dual_inf_tol", "compl_inf_tol", "acceptable_tol",
                              "acceptable_dual_inf_tol", "acceptable_compl_inf_tol"})
            opts->SetNumericValue(k, tol);
    }
    if (s.optim_constraint_tolerance != -1) {
        opts->SetNumericValue("constr_viol_tol", s.optim_constraint_tolerance);
        opts->SetNumericValue("acceptable_constr_viol_tol", s.optim_constraint_tolerance);
    }
}

class MocoHipTNLP : public Ipopt::TNLP {
public:
    using Index = Ipopt::Index;
    using Number = Ipopt::Number;

    // ctx: an mh_create'd context (unsharded, host entries).  guess: the
    // starting point on the transcription grid (e.g. a MocoTrajectory
    // resampled at the grid times, CasOCTranscription.cpp:593-597), or empty
    // for the bounds-midpoint guess (:1123-1149).
    explicit MocoHipTNLP(mh_ctx* ctx, std::vector<double> guess = {})
            : m_ctx(ctx), m_guess(std::move(guess)) {
        if (mh_get_nlp_info(m_ctx, &m_info) != MH_OK) throw std::runtime_error(mh_last_error());
        if (!m_guess.empty() && (int64_t)m_guess.size() != m_info.n)
            throw std::invalid_argument("guess size does not match the NLP");
    }

    bool get_nlp_info(Index& n, Index& m, Index& nnz_jac, Index& nnz_h, IndexStyleEnum& style) override {
        n = (Index)m_info.n;
        m = (Index)m_info.m;
        nnz_jac = (Index)m_info.nnz_jac_g;
        nnz_h = 0;                 // limited-memory Hessian approximation
        style = C_STYLE;           // 0-based, as mh_get_jac_structure
        return true;
    }
    bool get_bounds_info(Index, Number* xl, Number* xu, Index, Number* gl, Number* gu) override {
        return mh_get_bounds(m_ctx, xl, xu, gl, gu) == MH_OK;
    }
    bool get_starting_point(Index n, bool init_x, Number* x, bool init_z, Number*, Number*, Index,
            bool init_lambda, Number*) override {
        if (init_z || init_lambda) return false;   // no warm start (IPOPTSolver.cpp:357-372)
        if (!init_x) return true;
        if (m_guess.empty()) return mh_get_initial_guess_from_bounds(m_ctx, x) == MH_OK;
        std::copy(m_guess.begin(), m_guess.begin() + n, x);
        return true;
    }
    bool eval_f(Index, const Number* x, bool new_x, Number& f) override {
        return mh_eval_f(m_ctx, x, new_x, &f) == MH_OK;
    }
    bool eval_grad_f(Index, const Number* x, bool new_x, Number* grad) override {
        return mh_eval_grad_f(m_ctx, x, new_x, grad) == MH_OK;
    }
    bool eval_g(Index, const Number* x, bool new_x, Index, Number* g) override {
        return mh_eval_g(m_ctx, x, new_x, g) == MH_OK;
    }
    bool eval_jac_g(Index, const Number* x, bool new_x, Index, Index, Index* iRow, Index* jCol,
            Number* values) override {
        if (!values) {                                 // structure request
            static_assert(sizeof(Index) == sizeof(int32_t), "Ipopt::Index must be 32-bit");
            return mh_get_jac_structure(m_ctx, reinterpret_cast<int32_t*>(iRow),
                                        reinterpret_cast<int32_t*>(jCol)) == MH_OK;
        }
        return mh_eval_jac_g(m_ctx, x, new_x, values) == MH_OK;
    }
    void finalize_solution(Ipopt::SolverReturn status, Index n, const Number* x, const Number*,
            const Number*, Index, const Number*, const Number*, Number obj, const Ipopt::IpoptData* ip_data,
            Ipopt::IpoptCalculatedQuantities*) override {
        m_status = status;
        m_objective = obj;
        m_solution.assign(x, x + n);
        m_iterations = ip_data ? ip_data->iter_count() : -1;
    }

    const std::vector<double>& solution() const { return m_solution; }
    double objective() const { return m_objective; }
    int iterations() const { return m_iterations; }
    Ipopt::SolverReturn status() const { return m_status; }

private:
    mh_ctx* m_ctx;
    mh_nlp_info m_info{};
    std::vector<double> m_guess;
    std::vector<double> m_solution;
    double m_objective = 0.0;
    int m_iterations = -1;
    Ipopt::SolverReturn m_status = Ipopt::UNASSIGNED;
};

// One solve: create the Ipopt application, map the options, run.  Returns
// Ipopt's status; the solution iterate is in tnlp->solution() (convert it
// back to a MocoTrajectory at the grid times).
inline Ipopt::ApplicationReturnStatus solve(const Ipopt::SmartPtr<MocoHipTNLP>& tnlp,
        const IpoptSettings& settings) {
    Ipopt::SmartPtr<Ipopt::IpoptApplication> app = IpoptApplicationFactory();
    apply_ipopt_options(*app, settings);
    Ipopt::ApplicationReturnStatus st = app->Initialize();
    if (st != Ipopt::Solve_Succeeded) return st;
    return app->OptimizeTNLP(Ipopt::SmartPtr<Ipopt::TNLP>(GetRawPtr(tnlp)));
}

}  // namespace mocohip
