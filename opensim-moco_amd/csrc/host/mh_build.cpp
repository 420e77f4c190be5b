// mh_build.cpp — the native problem builder as a tool: an OpenSim-level
// description of a MocoStudy (mocohip/describe.py) -> the problem tape that
// mh_driver (and any C++ host over the C ABI) runs, lowered by mh_builder
// (compileProblemRep's rules in C++).
//
//   mh_build <description> <tape> [--shard BEGIN END] [--solution X.bin OUT.sto]
//
// --solution: the iterate X.bin (raw float64, the NLP's n) as the
// MocoSolution the plugin returns (mh_trajectory.hpp: every block by the
// reference's names), written as a .sto; the conversion back to an iterate
// must give X bit for bit ("roundtrip" in the JSON line).
//
// Prints one JSON line (state / control / goal counts); exit status 0 ok,
// 1 usage or input error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

#include <vector>

#include "mh_builder.hpp"
#include "mh_trajectory.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <description> <tape> [--shard BEGIN END]\n", argv[0]);
        return 1;
    }
    int ib = 0, ie = 0;
    const char *xbin = nullptr, *sto = nullptr;
    for (int a = 3; a < argc; ++a) {
        if (std::strcmp(argv[a], "--shard") == 0 && a + 2 < argc) {
            ib = std::atoi(argv[a + 1]);
            ie = std::atoi(argv[a + 2]);
            a += 2;
        } else if (std::strcmp(argv[a], "--solution") == 0 && a + 2 < argc) {
            xbin = argv[a + 1];
            sto = argv[a + 2];
            a += 2;
        } else {
            std::fprintf(stderr, "unknown argument %s\n", argv[a]);
            return 1;
        }
    }
    try {
        mhb::Problem P;
        mhb::SolverSettings S;
        mhb::read_description(argv[1], P, S);
        mhb::ProblemRep R;
        mhb::make_rep(P, R);
        const mh_options o = mhb::make_options(S, ib, ie);
        mhb::write_tape(R, o, argv[2]);
        std::string sol;
        if (xbin) {
            const mhb::IterateLayout L = mhb::iterate_layout(R, o);
            std::vector<double> x((size_t)L.n());
            FILE* f = std::fopen(xbin, "rb");
            if (!f) throw std::runtime_error(std::string("cannot read ") + xbin);
            const size_t got = std::fread(x.data(), sizeof(double), x.size(), f);
            const bool extra = std::fgetc(f) != EOF;
            std::fclose(f);
            if (got != x.size() || extra) throw std::runtime_error("the iterate's size is not the NLP's n");
            const mhb::TrajectoryTable T = mhb::iterate_to_trajectory(x, R, o);
            mhb::write_sto(T, sto);
            const std::vector<double> back = mhb::trajectory_to_iterate(T, R, o);
            const bool same = back.size() == x.size() &&
                              std::memcmp(back.data(), x.data(), sizeof(double) * x.size()) == 0;
            sol = std::string(", \"solution\": \"") + sto + "\", \"n\": " + std::to_string(L.n()) +
                  ", \"multipliers\": " + std::to_string(T.multiplier_names.size()) +
                  ", \"derivatives\": " + std::to_string(T.derivative_names.size()) +
                  ", \"slacks\": " + std::to_string(T.slack_names.size()) +
                  ", \"roundtrip\": " + (same ? "true" : "false");
        }
        std::printf("{\"tape\": \"%s\", \"nq\": %d, \"states\": %zu, \"controls\": %zu, \"goals\": %d, "
                    "\"path_equations\": %d, \"endpoint_equations\": %d, \"tables\": %d%s}\n",
                    argv[2], R.cm.model.nq, R.state_names.size(), R.control_names.size(), R.problem.ngoals,
                    R.problem.npath, R.problem.nendpoint, R.cm.model.ntables, sol.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "mh_build: %s\n", e.what());
        return 1;
    }
    return 0;
}
