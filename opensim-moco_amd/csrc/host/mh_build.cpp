// mh_build.cpp — the native problem builder as a tool: an OpenSim-level
// description of a MocoStudy (mocohip/describe.py) -> the problem tape that
// mh_driver (and any C++ host over the C ABI) runs, lowered by mh_builder
// (compileProblemRep's rules in C++).
//
//   mh_build <description> <tape> [--shard BEGIN END]
//
// Prints one JSON line (state / control / goal counts); exit status 0 ok,
// 1 usage or input error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

#include "mh_builder.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <description> <tape> [--shard BEGIN END]\n", argv[0]);
        return 1;
    }
    int ib = 0, ie = 0;
    for (int a = 3; a < argc; ++a) {
        if (std::strcmp(argv[a], "--shard") == 0 && a + 2 < argc) {
            ib = std::atoi(argv[a + 1]);
            ie = std::atoi(argv[a + 2]);
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
        std::printf("{\"tape\": \"%s\", \"nq\": %d, \"states\": %zu, \"controls\": %zu, \"goals\": %d, "
                    "\"path_equations\": %d, \"endpoint_equations\": %d, \"tables\": %d}\n",
                    argv[2], R.cm.model.nq, R.state_names.size(), R.control_names.size(), R.problem.ngoals,
                    R.problem.npath, R.problem.nendpoint, R.cm.model.ntables);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "mh_build: %s\n", e.what());
        return 1;
    }
    return 0;
}
