"""The C-ABI library loads, exports every entry point include/mocohip.h
declares, and the ctypes mirror matches the header's struct layout.  No
compute calls (CPU only)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from mocohip import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mocohip.h")
KKT_HEADER = os.path.join(ROOT, "include", "mocohip_kkt.h")

STRUCTS = ["mh_function", "mh_axis", "mh_body", "mh_path_point", "mh_muscle", "mh_spring",
           "mh_parameter_target",
           "mh_actuator", "mh_table", "mh_external_force", "mh_constraint", "mh_wrap_object",
           "mh_path_wrap", "mh_model",
           "mh_bounds", "mh_variable_info", "mh_goal", "mh_path_equation", "mh_endpoint_equation",
           "mh_problem",
           "mh_options", "mh_nlp_info"]


def header_functions(path=HEADER):
    src = open(path).read()
    return sorted(set(re.findall(r"\b(mh_[a-z_]+)\s*\(", src)) - set(STRUCTS))


def test_header_declares_exactly_the_bound_symbols():
    assert header_functions() == sorted(abi.MOCOHIP_SYMBOLS)
    assert header_functions(KKT_HEADER) == sorted(abi.MOCOHIP_KKT_SYMBOLS)


def test_library_loads_and_exports_every_symbol():
    lib = abi.load_mocohip()
    for name in list(abi.MOCOHIP_SYMBOLS) + list(abi.MOCOHIP_KKT_SYMBOLS):
        assert hasattr(lib, name), name
    assert lib.mh_abi_version() == abi.MH_ABI_VERSION == 8
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIBMOCOHIP_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mh_\w+)", out))
    assert set(abi.MOCOHIP_SYMBOLS) | set(abi.MOCOHIP_KKT_SYMBOLS) <= exported


@pytest.mark.parametrize("name", ["sliding_mass", "double_pendulum", "gait10dof18musc"])
def test_host_model_hash_matches_library(name):
    """tools/gen_models.py keys the generated back ends with abi.model_hash
    (host restatement); mh_create selects them with mh_model_hash."""
    from mocohip import configs
    lib = abi.load_mocohip()
    rep = configs.CONFIGS[name](4).problem.create_rep()
    h = C.c_uint64()
    assert lib.mh_model_hash(C.byref(rep.struct.model), C.byref(h)) == 0
    assert h.value == abi.model_hash(rep.struct.model)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", abi.LIBMOCOHIP_PATH],
                         capture_output=True, text=True)
    blob = open(abi.LIBMOCOHIP_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layout_matches_header():
    prog = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"',
            "int main(void) {"]
    for s in STRUCTS:
        prog.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for fname, _ in getattr(abi, s)._fields_:
            prog.append(f'printf("{s}.{fname} %zu\\n", offsetof({s}, {fname}));')
    prog += ["return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write("\n".join(prog))
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-std=c99", "-o", exe, c], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    want = dict(l.split() for l in out.splitlines())
    for s in STRUCTS:
        T = getattr(abi, s)
        assert int(want[s]) == C.sizeof(T), s
        for fname, _ in T._fields_:
            assert int(want[f"{s}.{fname}"]) == getattr(T, fname).offset, f"{s}.{fname}"


def test_no_cpu_fallback_without_gpu():
    """On a host without a gfx950 device, mh_create must fail loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mocohip import configs
    from mocohip.solver import HipNLP
    st = configs.sliding_mass(4)
    with pytest.raises(RuntimeError, match="no CPU fallback|HIP"):
        HipNLP(st.problem.create_rep(), st.solver.options())
