/* MocoHipSolver.h — the MocoSolver plugin that runs Moco's direct-collocation
 * hot path on an MI355X (libmocohip.so, include/mocohip.h).
 *
 * What a Moco user swaps: MocoStudy::initSolver<MocoHipSolver>() (or
 * <MocoHipSolver> in the study's <solver> XML property, MocoStudy.h:145-167)
 * instead of MocoCasADiSolver.  It derives from MocoDirectCollocationSolver
 * (MocoDirectCollocationSolver.h:86-170), so every property of that class --
 * num_mesh_intervals, transcription_scheme, interpolate_control_midpoints,
 * multibody_dynamics_mode, optim_* tolerances, kinematic-constraint options,
 * guess_file -- keeps its meaning; it adds MocoCasADiSolver's
 * optim_finite_difference_scheme and optim_sparsity_detection
 * (MocoCasADiSolver.h:115-159) and a HIP device ordinal.
 *
 * NOT compiled in this repository: OpenSim (opensim-core b0222c2 + Simbody
 * 3.7) and Ipopt 3.12.8 are absent from the build image.
 * It is written against their public headers; everything it calls on this
 * repository's side -- the C ABI, the C++ problem builder
 * (opensim-moco_amd/csrc/host/mh_builder.hpp) and the Ipopt TNLP adapter
 * (csrc/host/mh_ipopt_tnlp.hpp) -- is built and tested here
 * (tests/test_builder.py, tests/test_host_driver.py).  Registration:
 * Object::registerType(MocoHipSolver()) beside the other solvers in
 * RegisterTypes_osimMoco.cpp:68-150. */
#ifndef MOCOHIP_INTEGRATION_MOCOHIPSOLVER_H
#define MOCOHIP_INTEGRATION_MOCOHIPSOLVER_H

#include <OpenSim/Moco/MocoDirectCollocationSolver.h>

#include "mh_builder.hpp"

namespace OpenSim {

class MocoProblemRep;

/* compileProblemRep: the lowering of a MocoProblemRep (its model, variable
 * infos, goals, path constraints, kinematic constraints, prescribed
 * kinematics) into the builder's description, which mhb::make_rep turns into
 * the C-ABI mh_problem with the reference's ordering and default-bound rules
 * (Simbody Y order, MocoUtilities.cpp:495-528; MocoProblemRep.cpp:306-444).
 * Throws OpenSim::Exception for components outside the implemented path
 * (DESIGN.md §7): joints other than Custom / Pin / Slider / Weld / Free-less
 * trees, muscles other than DeGrooteFregly2016Muscle, wrap surfaces other
 * than WrapCylinder, goals outside SURVEY §8 A11. */
mhb::Problem compileProblemRep(const MocoProblemRep& rep);

class MocoHipSolver : public MocoDirectCollocationSolver {
    OpenSim_DECLARE_CONCRETE_OBJECT(MocoHipSolver, MocoDirectCollocationSolver);

public:
    OpenSim_DECLARE_PROPERTY(optim_finite_difference_scheme, std::string,
            "The finite difference scheme CasADi would use for the "
            "callbacks' derivatives: 'central' (default), 'forward' or "
            "'backward' (MocoCasADiSolver.h:123-127).");
    OpenSim_DECLARE_PROPERTY(optim_sparsity_detection, std::string,
            "'none' (block-dense, default), 'random' or 'initial-guess' "
            "(MocoCasADiSolver.h:129-137).");
    OpenSim_DECLARE_PROPERTY(device, int, "HIP device ordinal (default 0).");
    OpenSim_DECLARE_PROPERTY(jacobian_mode, std::string,
            "'callback-fd' (MocoCasADiSolver's Jacobian, default) or "
            "'global-seeds' (MocoTropterSolver's ColPack-seeded FD of g).");

    MocoHipSolver();

    /* The bounds-midpoint guess on this solver's grid
     * (CasOCTranscription.cpp:1123-1149), as a MocoTrajectory. */
    MocoTrajectory createGuess(const std::string& type = "bounds") const;
    void setGuess(MocoTrajectory guess);
    void setGuessFile(const std::string& file);
    const MocoTrajectory& getGuess() const;
    void clearGuess();

protected:
    void resetProblemImpl(const MocoProblemRep&) const override {}
    MocoSolution solveImpl() const override;

private:
    void constructProperties();
    mhb::SolverSettings settings() const;
    MocoTrajectory m_guessFromAPI;
    mutable SimTK::ResetOnCopy<MocoTrajectory> m_guessFromFile;
    mutable SimTK::ReferencePtr<const MocoTrajectory> m_guessToUse;
};

} // namespace OpenSim

#endif
