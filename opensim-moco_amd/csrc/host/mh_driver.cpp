// mh_driver.cpp — native C++ host over the C ABI (include/mocohip.h).
//
// What a C++ MocoSolver plugin / Ipopt::TNLP adapter does:
// load a compiled problem (a tape written by mocohip.tape.write_tape from a
// MocoProblemRep), create a context, and drive the NLP callbacks the way
// IPOPT does each iteration — eval_f, eval_grad_f, eval_g(new_x = true),
// eval_jac_g(new_x = false) — on host buffers (the TNLP contract; includes
// the PCIe transfer of g and the Jacobian values), then eval_g + eval_jac_g
// on device-resident buffers.  Prints one JSON line.
//
//   mh_driver <tape> [--steps K] [--warmup W] [--x x.bin] [--out gj.bin]
//
// --x: the iterate as raw float64 (default: mh_get_initial_guess_from_bounds)
// --out: writes g then the Jacobian values of the device path (raw float64)
// Exit status: 0 ok, 1 usage / tape error, 2 C-ABI error (e.g. no gfx950).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/mocohip.h"

namespace {

struct Reader {
    std::vector<char> buf;
    size_t pos = 0;
    bool ok = true;
    template <class T>
    T pod() {
        T v{};
        if (pos + sizeof(T) > buf.size()) { ok = false; return v; }
        std::memcpy(&v, buf.data() + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
    // n raw bytes (a zeroed buffer past the end, with ok cleared)
    const char* take(size_t n) {
        static std::vector<char> zero;
        if (pos + n > buf.size()) { ok = false; zero.assign(n, 0); return zero.data(); }
        const char* p = buf.data() + pos;
        pos += n;
        return p;
    }
    template <class T>
    std::vector<T> array(int64_t expected_count) {
        const int64_t bytes = pod<int64_t>();
        std::vector<T> v;
        if (!ok || bytes < 0 || bytes != expected_count * (int64_t)sizeof(T) ||
                pos + (size_t)bytes > buf.size()) {
            ok = false;
            return v;
        }
        v.resize((size_t)expected_count);
        if (bytes) std::memcpy(v.data(), buf.data() + pos, (size_t)bytes);
        pos += (size_t)bytes;
        return v;
    }
};

// A problem tape (mocohip/tape.py): owns the arrays mh_problem points into.
struct Tape {
    mh_options opts{};
    int ns = 0, nc = 0;
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
    std::vector<mh_variable_info> sinfo, cinfo;
    std::vector<mh_goal> goals;
    std::vector<int32_t> gidx, gcol;
    std::vector<double> gw;
    std::vector<mh_path_equation> path;
    std::vector<mh_endpoint_equation> endpoint;
    std::vector<mh_constraint> constraints;
    std::vector<mh_wrap_object> wraps;
    std::vector<mh_path_wrap> pathwraps;
    std::vector<mh_spring> springs;
    std::vector<mh_bounds> par_bounds;
    std::vector<mh_parameter_target> par_targets;
    std::vector<double> guess;
    std::vector<uint8_t> pattern;
    std::vector<int32_t> kin_col;
    mh_problem prob{};
};

bool read_tape(const char* path, Tape& t, std::string& err) {
    Reader r;
    FILE* f = std::fopen(path, "rb");
    if (!f) { err = std::string("cannot open ") + path; return false; }
    std::fseek(f, 0, SEEK_END);
    const long size = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    r.buf.resize(size > 0 ? (size_t)size : 0);
    const size_t got = r.buf.empty() ? 0 : std::fread(r.buf.data(), 1, r.buf.size(), f);
    std::fclose(f);
    if (got != r.buf.size() || r.buf.size() < 8 || std::memcmp(r.buf.data(), "MHTAPE01", 8) != 0) {
        err = "not a problem tape (magic MHTAPE01)";
        return false;
    }
    r.pos = 8;
    const int version = r.pod<int32_t>();
    t.ns = r.pod<int32_t>();
    t.nc = r.pod<int32_t>();
    // version 4 = ABI v4's mh_options (unchanged in v5); earlier tapes carry a
    // shorter one; version 5 appends the wrap surfaces; version 6 carries ABI
    // v6's mh_options (+ sparsity_rule: 8 bytes; older tapes leave it 0, the
    // reference's rule since v7); version 7: ABI v7 (the rule's values
    // swapped: a v6 tape's 0 / 1 was robust / any-change); version 8: ABI v8
    // (coloring_order in mh_options' former reserved word; the springs and
    // the MocoParameters appended; the initial-guess blob is the whole
    // iterate, n doubles)
    if (version < 4 || version > 8) {
        err = "unsupported tape version (this build reads versions 4 to 8)";
        return false;
    }
    {
        const size_t nopt = version >= 6 ? sizeof(mh_options) : sizeof(mh_options) - 2 * sizeof(int32_t);
        t.opts = mh_options{};
        std::memcpy(&t.opts, r.take(nopt), nopt);
        if (version == 6)
            t.opts.sparsity_rule = t.opts.sparsity_rule == 0 ? MH_SPARSITY_RULE_ROBUST : MH_SPARSITY_RULE_ANY_CHANGE;
    }
    mh_model& m = t.prob.model;
    int32_t* counts[] = {&m.nq, &m.nbodies, &m.naxes, &m.nfunctions, &m.nknots, &m.nmuscles,
                         &m.npoints, &m.nactuators, &m.ntables, &m.nbreaks, &m.ncoefs, &m.nexternal};
    for (int32_t* c : counts) *c = r.pod<int32_t>();
    for (double& g : m.gravity) g = r.pod<double>();
    t.prob.time_initial = r.pod<mh_bounds>();
    t.prob.time_final = r.pod<mh_bounds>();
    t.prob.ngoals = r.pod<int32_t>();
    t.prob.nterms = r.pod<int32_t>();
    t.bodies = r.array<mh_body>(m.nbodies);
    t.axes = r.array<mh_axis>(m.naxes);
    t.functions = r.array<mh_function>(m.nfunctions);
    t.knot_x = r.array<double>(m.nknots);
    t.knot_y = r.array<double>(m.nknots);
    t.muscles = r.array<mh_muscle>(m.nmuscles);
    t.points = r.array<mh_path_point>(m.npoints);
    t.actuators = r.array<mh_actuator>(m.nactuators);
    t.tables = r.array<mh_table>(m.ntables);
    t.breaks = r.array<double>(m.nbreaks);
    t.coefs = r.array<double>(m.ncoefs);
    t.external = r.array<mh_external_force>(m.nexternal);
    t.sinfo = r.array<mh_variable_info>(t.ns);
    t.cinfo = r.array<mh_variable_info>(t.nc);
    t.goals = r.array<mh_goal>(t.prob.ngoals);
    t.gidx = r.array<int32_t>(t.prob.nterms);
    t.gcol = r.array<int32_t>(t.prob.nterms);
    t.gw = r.array<double>(t.prob.nterms);
    if (version >= 2) {   // path-constraint equations
        t.prob.npath = r.pod<int32_t>();
        t.path = r.array<mh_path_equation>(t.prob.npath);
        const int64_t gbytes = r.pod<int64_t>();   // sparsity-detection guess
        if (r.ok && gbytes >= 0 && gbytes % 8 == 0 && r.pos + (size_t)gbytes <= r.buf.size()) {
            t.guess.resize((size_t)gbytes / 8);
            if (gbytes) std::memcpy(t.guess.data(), r.buf.data() + r.pos, (size_t)gbytes);
            r.pos += (size_t)gbytes;
        } else {
            r.ok = false;
        }
        const int64_t pbytes = r.pod<int64_t>();   // given callback sparsity
        if (r.ok && pbytes >= 0 && r.pos + (size_t)pbytes <= r.buf.size()) {
            t.pattern.assign(r.buf.data() + r.pos, r.buf.data() + r.pos + pbytes);
            r.pos += (size_t)pbytes;
        } else {
            r.ok = false;
        }
        t.prob.prescribed_kinematics = r.pod<int32_t>();   // prescribed kinematics
        t.prob.kinematics_table = r.pod<int32_t>();
        t.kin_col = r.array<int32_t>(t.prob.prescribed_kinematics ? m.nq : 0);
    }
    if (version >= 3) {   // endpoint-constraint equations
        t.prob.nendpoint = r.pod<int32_t>();
        t.endpoint = r.array<mh_endpoint_equation>(t.prob.nendpoint);
    }
    if (version >= 4) {   // kinematic constraints, multiplier / kinematic-row bounds
        m.nconstraints = r.pod<int32_t>();
        t.constraints = r.array<mh_constraint>(m.nconstraints);
        t.prob.multiplier_bounds = r.pod<mh_bounds>();
        t.prob.kinematic_constraint_bounds = r.pod<mh_bounds>();
    }
    if (version >= 5) {   // wrap surfaces and PathWraps
        m.nwraps = r.pod<int32_t>();
        t.wraps = r.array<mh_wrap_object>(m.nwraps);
        m.npathwraps = r.pod<int32_t>();
        t.pathwraps = r.array<mh_path_wrap>(m.npathwraps);
    }
    if (version >= 8) {   // springs, MocoParameters
        m.nsprings = r.pod<int32_t>();
        t.springs = r.array<mh_spring>(m.nsprings);
        t.prob.nparameters = r.pod<int32_t>();
        t.par_bounds = r.array<mh_bounds>(t.prob.nparameters);
        t.prob.nparameter_targets = r.pod<int32_t>();
        t.par_targets = r.array<mh_parameter_target>(t.prob.nparameter_targets);
    }
    if (!r.ok || r.pos != r.buf.size()) { err = "truncated or malformed tape"; return false; }
    m.bodies = t.bodies.data(); m.axes = t.axes.data(); m.functions = t.functions.data();
    m.knot_x = t.knot_x.data(); m.knot_y = t.knot_y.data(); m.muscles = t.muscles.data();
    m.points = t.points.data(); m.actuators = t.actuators.data(); m.tables = t.tables.data();
    m.table_breaks = t.breaks.data(); m.table_coefs = t.coefs.data(); m.external = t.external.data();
    t.prob.state_infos = t.sinfo.data();
    t.prob.control_infos = t.cinfo.data();
    t.prob.goals = t.goals.data();
    t.prob.goal_index = t.gidx.data();
    t.prob.goal_column = t.gcol.data();
    t.prob.goal_weight = t.gw.data();
    t.prob.path = t.path.data();
    t.opts.sparsity_guess = t.guess.empty() ? nullptr : t.guess.data();
    t.opts.sparsity_pattern = t.pattern.empty() ? nullptr : t.pattern.data();
    t.prob.kinematics_column = t.kin_col.empty() ? nullptr : t.kin_col.data();
    t.prob.endpoint = t.endpoint.empty() ? nullptr : t.endpoint.data();
    m.constraints = t.constraints.empty() ? nullptr : t.constraints.data();
    m.wraps = t.wraps.empty() ? nullptr : t.wraps.data();
    m.pathwraps = t.pathwraps.empty() ? nullptr : t.pathwraps.data();
    m.springs = t.springs.empty() ? nullptr : t.springs.data();
    t.prob.parameter_bounds = t.par_bounds.empty() ? nullptr : t.par_bounds.data();
    t.prob.parameter_targets = t.par_targets.empty() ? nullptr : t.par_targets.data();
    // the initial-guess iterate must be the whole x (mh_options.sparsity_guess:
    // n doubles, read by mh_create): sized against the host-only layout query
    if (!t.guess.empty()) {
        mh_nlp_info info{};
        if (mh_get_nlp_info_for(&t.prob, &t.opts, &info) != MH_OK) {
            err = std::string("tape problem rejected: ") + mh_last_error();
            return false;
        }
        if ((int64_t)t.guess.size() != info.n) {
            err = "the tape's initial-guess iterate has " + std::to_string(t.guess.size()) + " doubles, the "
                  "problem has n = " + std::to_string(info.n);
            return false;
        }
    }
    return true;
}

int fail_abi(const char* what, int rc) {
    std::fprintf(stderr, "mh_driver: %s failed (%d): %s\n", what, rc, mh_last_error());
    return 2;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: mh_driver <tape> [--steps K] [--warmup W] [--x x.bin] [--out gj.bin]\n");
        return 1;
    }
    int steps = 200, warmup = 20;
    const char* xpath = nullptr;
    const char* outpath = nullptr;
    for (int a = 2; a + 1 < argc; a += 2) {
        if (!std::strcmp(argv[a], "--steps")) steps = std::atoi(argv[a + 1]);
        else if (!std::strcmp(argv[a], "--warmup")) warmup = std::atoi(argv[a + 1]);
        else if (!std::strcmp(argv[a], "--x")) xpath = argv[a + 1];
        else if (!std::strcmp(argv[a], "--out")) outpath = argv[a + 1];
        else { std::fprintf(stderr, "mh_driver: unknown option %s\n", argv[a]); return 1; }
    }
    Tape tape;
    std::string err;
    if (!read_tape(argv[1], tape, err)) { std::fprintf(stderr, "mh_driver: %s\n", err.c_str()); return 1; }
    mh_ctx* ctx = nullptr;
    int rc = mh_create(&tape.prob, &tape.opts, &ctx);
    if (rc) return fail_abi("mh_create", rc);
    mh_nlp_info info;
    if ((rc = mh_get_nlp_info(ctx, &info))) return fail_abi("mh_get_nlp_info", rc);
    const size_t n = (size_t)info.n, m = (size_t)(info.row_end - info.row_begin),
                 nnz = (size_t)(info.nnz_end - info.nnz_begin);
    std::vector<double> x(n), g(m), v(nnz), grad(n);
    if (xpath) {
        FILE* f = std::fopen(xpath, "rb");
        if (!f || std::fread(x.data(), sizeof(double), n, f) != n) {
            std::fprintf(stderr, "mh_driver: cannot read %zu doubles from %s\n", n, xpath);
            return 1;
        }
        std::fclose(f);
    } else if ((rc = mh_get_initial_guess_from_bounds(ctx, x.data()))) {
        return fail_abi("mh_get_initial_guess_from_bounds", rc);
    }

    // IPOPT iteration on host buffers (TNLP): f, grad f, g(new_x), J(!new_x)
    double f = 0.0;
    auto ipopt_iter = [&]() -> int {
        int r;
        if ((r = mh_eval_f(ctx, x.data(), 1, &f))) return r;
        if ((r = mh_eval_grad_f(ctx, x.data(), 0, grad.data()))) return r;
        if ((r = mh_eval_g(ctx, x.data(), 0, g.data()))) return r;
        return mh_eval_jac_g(ctx, x.data(), 0, v.data());
    };
    for (int i = 0; i < warmup; ++i)
        if ((rc = ipopt_iter())) return fail_abi("host-pointer evaluation", rc);
    double t0 = now_s();
    for (int i = 0; i < steps; ++i)
        if ((rc = ipopt_iter())) return fail_abi("host-pointer evaluation", rc);
    const double host_s = now_s() - t0;

    // eval_g + eval_jac_g on device-resident buffers
    double *dx = nullptr, *dg = nullptr, *dv = nullptr;
    if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess || hipMalloc(&dg, sizeof(double) * (m + 1)) != hipSuccess ||
            hipMalloc(&dv, sizeof(double) * (nnz + 1)) != hipSuccess) {
        std::fprintf(stderr, "mh_driver: hipMalloc failed\n");
        return 2;
    }
    if (hipMemcpy(dx, x.data(), sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) return 2;
    auto dev_step = [&]() -> int {
        int r;
        if ((r = mh_eval_g_device(ctx, dx, dg))) return r;
        return mh_eval_jac_g_device(ctx, dx, dv);
    };
    for (int i = 0; i < warmup; ++i)
        if ((rc = dev_step())) return fail_abi("device-pointer evaluation", rc);
    t0 = now_s();
    for (int i = 0; i < steps; ++i)
        if ((rc = dev_step())) return fail_abi("device-pointer evaluation", rc);
    const double dev_s = now_s() - t0;
    // the same asynchronously (entries return once enqueued; one
    // synchronize at the end), separate and fused (mh_eval_g_jac_g_device)
    if ((rc = mh_set_async(ctx, 1))) return fail_abi("mh_set_async", rc);
    auto timed_async = [&](bool fused, double& secs) -> int {
        int r = 0;
        for (int i = 0; i < warmup && !r; ++i)
            r = fused ? mh_eval_g_jac_g_device(ctx, dx, dg, dv) : dev_step();
        if (!r) r = mh_synchronize(ctx);
        const double ta = now_s();
        for (int i = 0; i < steps && !r; ++i)
            r = fused ? mh_eval_g_jac_g_device(ctx, dx, dg, dv) : dev_step();
        if (!r) r = mh_synchronize(ctx);
        secs = now_s() - ta;
        return r;
    };
    double async_s = 0.0, fused_s = 0.0;
    if ((rc = timed_async(false, async_s))) return fail_abi("async device evaluation", rc);
    if ((rc = timed_async(true, fused_s))) return fail_abi("async fused device evaluation", rc);
    if ((rc = mh_set_async(ctx, 0))) return fail_abi("mh_set_async", rc);
    if (outpath) {
        std::vector<double> gd(m), vd(nnz);
        if (hipMemcpy(gd.data(), dg, sizeof(double) * m, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(vd.data(), dv, sizeof(double) * nnz, hipMemcpyDeviceToHost) != hipSuccess)
            return 2;
        FILE* fo = std::fopen(outpath, "wb");
        if (!fo) return 1;
        std::fwrite(gd.data(), sizeof(double), m, fo);
        std::fwrite(vd.data(), sizeof(double), nnz, fo);
        std::fclose(fo);
    }
    char be[128] = {0};
    double fl = 0.0;
    uint64_t hash = 0;
    mh_get_backend(ctx, be, sizeof be, &fl, &hash);
    std::printf("{\"driver\": \"mh_driver (C++ host over the C ABI)\", \"backend\": \"%s\", \"n\": %lld, "
                "\"m\": %lld, \"nnz\": %lld, \"steps\": %d, "
                "\"ipopt_iteration_host_pointers_per_s\": %.3f, "
                "\"eval_g_jac_g_device_pointers_per_s\": %.3f, "
                "\"async_separate_per_s\": %.3f, \"async_fused_per_s\": %.3f, \"f\": %.17g}\n",
                be, (long long)info.n, (long long)info.m, (long long)info.nnz_jac_g, steps, steps / host_s,
                steps / dev_s, steps / async_s, steps / fused_s, f);
    (void)hipFree(dx);
    (void)hipFree(dg);
    (void)hipFree(dv);
    mh_destroy(ctx);
    return 0;
}
