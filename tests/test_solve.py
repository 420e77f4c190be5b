"""End to end: MocoStudy.solve() on the GPU path (HipNLP) with the host NLP
driver (mocohip.nlpsolve; Ipopt is absent), against the reference's own
known-answer tests of whole solves."""
import numpy as np
import pytest

from mocohip import configs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scheme,dynamics", [("trapezoidal", "explicit"), ("trapezoidal", "implicit"),
                                             ("hermite-simpson", "explicit")])
def test_sliding_mass_known_solution(scheme, dynamics):
    """testMocoInterface.cpp:1701-1742 ("Sliding mass"): bang-bang control,
    final time 2.0, position and speed the quadratic / triangle profiles,
    force +-10, all within the reference's 1e-2; the reference's state and
    control names.  Also in implicit dynamics mode (testImplicit.cpp solves
    its problems in both modes) and with Hermite-Simpson."""
    sol = configs.sliding_mass_interface(scheme=scheme, dynamics=dynamics).solve()
    assert sol.metadata["success"] == "true", sol.metadata
    assert sol.state_names == ["/slider/position/value", "/slider/position/speed"]
    assert sol.control_names == ["/actuator"]
    t = sol.time
    assert len(t) == (20 if scheme == "trapezoidal" else 39)
    assert t[-1] == pytest.approx(2.0, abs=1e-2)
    half = 0.5 * t[-1]
    pos = np.where(t < half, 0.5 * t ** 2, -0.5 * (t - half) ** 2 + (t - half) + 0.5)
    spd = np.where(t < half, t, t[-1] - t)
    frc = np.where(t < half, 10.0, -10.0)
    mesh = np.arange(len(t)) % (1 if scheme == "trapezoidal" else 2) == 0
    # (Hermite-Simpson: the midpoint of the interval holding the switch
    # sits on the speed peak, which the cubic interpolant cuts by ~0.026)
    near = (~mesh) & (np.abs(t - half) < 0.06)
    assert np.abs(sol.states[:, 0] - pos).max() < 1e-2
    assert np.abs(sol.states[~near, 1] - spd[~near]).max() < 1e-2
    # the switch is inside one mesh interval: compare the force away from it
    away = mesh & (np.abs(t - half) > 0.15)
    assert np.abs(sol.controls[away, 0] - frc[away]).max() < 1e-2
