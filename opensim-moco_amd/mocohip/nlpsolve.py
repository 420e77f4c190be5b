"""A host NLP driver over the C ABI's TNLP-shaped entries.

MocoCasADiSolver hands the transcription to Ipopt (MocoCasADiSolver.cpp:
210-260; tropter: IPOPTSolver.cpp:302-447); Ipopt 3.12.8 is not in this
image, so ``solve_nlp`` drives the same callbacks -- bounds, eval_f,
eval_grad_f, eval_g, eval_jac_g with the fixed sparse structure -- with
``method``:

  "ipm" (default)   mocohip.ipm: the primal-dual interior-point filter
                    line-search algorithm Ipopt implements, with its
                    limited-memory BFGS Hessian (the reference's
                    hessian_approximation = limited-memory,
                    MocoDirectCollocationSolver.cpp:35) and Ipopt's
                    termination options;
  "SLSQP", "trust-constr"   scipy's optimizers (dense SQP / trust region),
                    kept for comparison.

These are substitute optimizers, not Ipopt: iterate sequences differ;
converged solutions of well-posed problems agree to the tolerances.  Every
function and derivative evaluation goes through the NLP object it is given
(HipNLP: the GPU path)."""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class NLPResult:
    x: np.ndarray
    success: bool
    status: str
    objective: float
    iterations: int
    duration: float          # wall-clock seconds of the solve
    constraint_violation: float   # unscaled max bound violation of g at x
    evaluations: dict
    optimizer: str = ""
    timings: Optional[dict] = None
    history: Optional[list] = None


def solve_nlp(nlp, x0: np.ndarray, tol: float = 1e-8, constraint_tol: float = 1e-8,
              max_iter: int = 5000, verbose: int = 0, method: str = "ipm",
              ipopt_options: Optional[dict] = None) -> NLPResult:
    """Minimize nlp.eval_f subject to the NLP's bounds from x0.

    ipopt_options (method "ipm"): Ipopt option names (MocoHipSolver.
    ipopt_options(): tol, dual_inf_tol, compl_inf_tol, constr_viol_tol,
    acceptable_*, max_iter, print_level); when None, ``tol`` sets tol /
    dual_inf_tol / compl_inf_tol and ``constraint_tol`` constr_viol_tol."""
    if method == "ipm":
        from .ipm import IpmOptions, solve_ipm
        if ipopt_options is None:
            ipopt_options = {"tol": tol, "dual_inf_tol": tol, "compl_inf_tol": tol,
                             "acceptable_tol": tol, "acceptable_dual_inf_tol": tol,
                             "acceptable_compl_inf_tol": tol, "constr_viol_tol": constraint_tol,
                             "acceptable_constr_viol_tol": constraint_tol, "max_iter": max_iter}
        opts = IpmOptions.from_ipopt(ipopt_options)
        if verbose:
            opts.print_level = 1
        r = solve_ipm(nlp, x0, opts)
        return NLPResult(r.x, r.success, r.status, r.objective, r.iterations, r.duration,
                         r.constraint_violation, r.evaluations, "mocohip.ipm (interior point, L-BFGS)",
                         r.timings, r.history)
    return _solve_scipy(nlp, x0, tol, constraint_tol, max_iter, verbose, method)


def _solve_scipy(nlp, x0, tol, constraint_tol, max_iter, verbose, method):
    from scipy.optimize import BFGS, Bounds, NonlinearConstraint, minimize
    from scipy.sparse import csr_matrix
    if method == "auto":
        method = "SLSQP" if nlp.n * max(nlp.m, 1) <= 4_000_000 else "trust-constr"
    if method not in ("SLSQP", "trust-constr"):
        raise ValueError(f"unknown method {method!r}")
    n, m = nlp.n, nlp.m
    xl, xu, gl, gu = nlp.bounds()
    xl, xu = np.asarray(xl[:n], float), np.asarray(xu[:n], float)
    gl, gu = np.asarray(gl[:m], float), np.asarray(gu[:m], float)
    ir, jc = nlp.jac_structure()
    ir, jc = np.asarray(ir[:nlp.nnz]), np.asarray(jc[:nlp.nnz])
    counts = {"f": 0, "grad_f": 0, "g": 0, "jac_g": 0}

    def f(x):
        counts["f"] += 1
        return float(nlp.eval_f(x))

    def grad_f(x):
        counts["grad_f"] += 1
        return nlp.eval_grad_f(x)

    def g(x):
        counts["g"] += 1
        return nlp.eval_g(x)[:m]

    def jac_g(x):
        counts["jac_g"] += 1
        return csr_matrix((nlp.eval_jac_g(x)[:nlp.nnz], (ir, jc)), shape=(m, n))

    x0 = np.clip(np.asarray(x0, float), xl, xu)
    t0 = time.perf_counter()
    if method == "SLSQP":
        eq = np.where(gl == gu)[0]
        lo = np.where((gl != gu) & np.isfinite(gl))[0]
        up = np.where((gl != gu) & np.isfinite(gu))[0]
        cache = {}

        def gj(x):   # one g and one Jacobian per iterate, shared by the rows
            k = x.tobytes()
            if cache.get("k") != k:
                cache.update(k=k, g=g(x), J=jac_g(x).toarray())
            return cache["g"], cache["J"]
        cons = []
        if len(eq):
            cons.append({"type": "eq", "fun": lambda x: gj(x)[0][eq] - gl[eq], "jac": lambda x: gj(x)[1][eq]})
        if len(lo):
            cons.append({"type": "ineq", "fun": lambda x: gj(x)[0][lo] - gl[lo], "jac": lambda x: gj(x)[1][lo]})
        if len(up):
            cons.append({"type": "ineq", "fun": lambda x: gu[up] - gj(x)[0][up], "jac": lambda x: -gj(x)[1][up]})
        res = minimize(f, x0, jac=grad_f, method="SLSQP", bounds=Bounds(xl, xu), constraints=cons,
                       options={"ftol": tol, "maxiter": max_iter, "disp": bool(verbose)})
        converged = res.status == 0
    else:
        cons = [NonlinearConstraint(g, gl, gu, jac=jac_g, hess=BFGS())] if m else []
        res = minimize(f, x0, jac=grad_f, hess=BFGS(), method="trust-constr", bounds=Bounds(xl, xu),
                       constraints=cons,
                       options={"gtol": tol, "xtol": 1e-12, "barrier_tol": tol, "maxiter": max_iter,
                                "verbose": verbose})
        converged = res.status in (1, 2)
    el = time.perf_counter() - t0
    gx = nlp.eval_g(res.x)[:m]
    viol = float(np.max(np.concatenate([[0.0], gl - gx, gx - gu]))) if m else 0.0
    # absolute violation bound, like Ipopt's constr_viol_tol (no scaling by |g|)
    ok = bool(converged and viol <= max(constraint_tol, 1e-6))
    return NLPResult(res.x, ok, f"{method}: {res.message}", float(res.fun), int(res.nit), el, viol,
                     counts, f"scipy {method}")
