"""Host-side checks of the model-specialized code generator's task
decomposition (codegen.py): the subtree split of the mass-matrix and RNEA
groups.  The numerics of the emitted code are checked on the GPU against
the oracle (tests/test_gpu_parity.py); here: that every quantity the
single-lane DAE computes has exactly one producer among the groups."""
import pytest

from mocohip import codegen, configs
from mocohip.codegen import ModelView, branch_parts, coordinate_tree, generate


def _model(study):
    rep = study.problem.create_rep()
    codegen._CTX = codegen._Ctx()
    return rep, ModelView(rep.compiled)


def _coord_body(M):
    E = codegen._Emitter(M, codegen._Layout(M))
    return E.kinematics(list(range(M.nb)), accel=False, vel=False)[5]


@pytest.mark.parametrize("mk", [lambda: configs.gait10dof18musc(4), lambda: configs.rajagopal80(4)])
def test_branch_parts_partition_the_tree(mk):
    rep, M = _model(mk())
    root, parts = branch_parts(M)
    assert root == [0]                                   # the pelvis
    assert len(parts) == 3                               # two legs and the torso
    every = sorted(b for p in parts for b in p)
    assert every == list(range(M.nb))                    # each body in exactly one part
    for p in parts:                                      # parts are subtrees (+ the root chain)
        for b in p:
            assert M.bodies[b].parent in p or M.bodies[b].parent in root or M.bodies[b].parent < 0


def test_chains_are_not_split():
    _, M = _model(configs.double_pendulum(4))
    assert branch_parts(M) is None
    src, info = generate(_model(configs.double_pendulum(4))[0].compiled, "X")
    assert [g[0] for g in info["groups"]][:2] == ["mass", "bias"]


@pytest.mark.parametrize("mk,implicit,prescribed", [
    (lambda: configs.gait10dof18musc(4), False, False),
    (lambda: configs.gait10dof18musc(4, tendon_compliance=True), False, False),
    (lambda: configs.rajagopal80(4), False, False),
    (lambda: configs.gait10dof18musc_inverse(4), True, True),
])
def test_split_groups_cover_the_dae_once(mk, implicit, prescribed):
    rep, M = _model(mk())
    codegen._CTX = codegen._Ctx()
    cb = _coord_body(M)
    lam = coordinate_tree(M, cb, M.nq)
    root, parts = branch_parts(M)
    codegen._CTX = None
    src, info = generate(rep.compiled, "X", implicit=implicit, prescribed=prescribed)
    groups = info["groups"]
    names = [g[0] for g in groups]
    assert names[0] == "mass"                            # the placeholder keeps its slot
    if not implicit:
        # the mass-matrix parts: every factor entry of a non-root coordinate
        # from exactly one part, every root-chain entry shared by each part
        want = {(i, j) for i in range(M.nq) for j in [i] + _ancestors(lam, i)}
        root_coords = {j for j in cb if cb[j] in root}
        own = [k for k in want if k[0] not in root_coords]
        nparts = sum(1 for n in names if n.startswith("mass_"))
        assert nparts == len(parts)
        codegen._CTX = codegen._Ctx()
        gs = codegen._emit_groups(M, codegen._Layout(M, implicit, prescribed))
        codegen._CTX = None
        H = [k for g in gs if g.name.startswith("mass_") for kind, k in g.fields if kind == "H"]
        HR = [k for g in gs if g.name.startswith("mass_") for kind, k in g.fields if kind == "HR"]
        assert sorted(H) == sorted(own)                  # each factor entry once
        shared = sorted(k for k in want if k[0] in root_coords)
        assert sorted(HR) == sorted(shared * nparts)     # each part's share of the root block
        # a part reads its own subtree's and the root chain's coordinates only
        for g in gs:
            if g.name.startswith("mass_"):
                own_q = {k[0] for kind, k in g.fields if kind == "H"} | root_coords
                assert set(g.reads) <= own_q
    assert sum(1 for n in names if n.startswith("bias_")) == len(parts)
    assert f"NHEAVY = {1 + sum(1 for n in names if n.startswith(('mass_', 'bias_')))}" in src
    for im in range(len(M.muscles)):
        assert f"muscle_{im}" in names


def _ancestors(lam, i):
    out, j = [], lam[i]
    while j >= 0:
        out.append(j)
        j = lam[j]
    return out
