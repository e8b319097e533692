"""C-ABI checks that need no GPU: the library loads, exports every entry point
include/sphcore.h declares, the ctypes PODs match the C layout, and the core's
constant derivation (JSph::ConfigConstants1/2) agrees with the oracle's."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from dualsphysics_multilayer_amd import _abi
from dualsphysics_multilayer_amd.case import DamBreakCase
from dualsphysics_multilayer_amd.core import EXPORTED_SYMBOLS, LIB_PATH, case_derive, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sphcore.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sph_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB_PATH), "libsphcore.so not built"
    L = C.CDLL(LIB_PATH)
    decl = declared_functions()
    assert decl, "no declarations parsed"
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(EXPORTED_SYMBOLS) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    for name in decl:
        assert re.search(r"\bT %s$" % name, out, re.M), name


def test_abi_version_and_error_channel():
    L = load_library()
    assert L.sph_abi_version() == _abi.SPH_ABI_VERSION
    # Invalid arguments are rejected with SPH_ERR_ARG and a message, no crash.
    assert L.sph_solver_run(None, 1) == 1
    assert b"invalid argument" in L.sph_last_error()


def test_struct_layouts_match_c(tmp_path):
    prog = tmp_path / "sizes.c"
    prog.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
        "int main(){printf(\"%%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n\",sizeof(SphCaseDef),sizeof(SphConstants),"
        "sizeof(SphRunStats),sizeof(SphParticlesHost),sizeof(SphInterOut),offsetof(SphCaseDef,npb),"
        "offsetof(SphConstants,dom_cellcode),sizeof(SphSlabDef),offsetof(SphSlabDef,comm_id),sizeof(SphPartHeader),offsetof(SphPartHeader,pos_double));return 0;}\n" % HEADER
    )
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", str(prog), "-o", str(exe)])
    got = list(map(int, subprocess.check_output([str(exe)]).split()))
    py = [
        C.sizeof(_abi.SphCaseDef),
        C.sizeof(_abi.SphConstants),
        C.sizeof(_abi.SphRunStats),
        C.sizeof(_abi.SphParticlesHost),
        C.sizeof(_abi.SphInterOut),
        _abi.SphCaseDef.npb.offset,
        _abi.SphConstants.dom_cellcode.offset,
        C.sizeof(_abi.SphSlabDef),
        _abi.SphSlabDef.comm_id.offset,
        C.sizeof(_abi.SphPartHeader),
        _abi.SphPartHeader.pos_double.offset,
    ]
    assert got == py


@pytest.mark.parametrize("dp", [0.02, 0.0127, 0.0045])
def test_derived_constants_match_oracle(dp):
    oracle = pytest.importorskip("oracle.pyoracle")
    cdef = DamBreakCase(dp).case_def()
    a = case_derive(cdef)
    b = oracle.derive(cdef)
    assert a == b


def test_derived_constants_match_reference_log():
    # Values printed by the reference solver's Run.out for the dp=0.02 case
    # (JSph::VisuConfig): Cs0, DtIni, DtMin, MapCells, DomCellCode "1+11_10_10".
    k = case_derive(DamBreakCase(0.02).case_def())
    assert k["cs0"] == pytest.approx(34.31034761008696, rel=0, abs=1e-12)
    assert k["dtini"] == pytest.approx(0.001009637578387765, rel=1e-15)
    assert k["dtmin"] == pytest.approx(5.048187967162685e-05, rel=1e-15)
    assert k["dom_cells"] == [24, 10, 9]
    dcc = k["dom_cellcode"]
    assert ((dcc >> 25) - 1, (dcc >> 20) & 31, (dcc >> 15) & 31) == (11, 10, 10)


def test_invalid_case_rejected():
    cdef = DamBreakCase(0.05).case_def()
    cdef["kernel"] = 3  # TpKernel: 1 Cubic, 2 Wendland (JSph.cpp:554-559)
    with pytest.raises(RuntimeError, match="Kernel choice"):
        case_derive(cdef)


def test_cubic_constants():
    """GetKernelCubic_Ctes (FunSphKernel.h:51-84), 3-D and 2-D."""
    import math

    from dualsphysics_multilayer_amd.case import DamBreak2DCase

    for c in (DamBreakCase(0.05, kernel=1), DamBreak2DCase(0.05, kernel=1)):
        k = case_derive(c.case_def())
        h = float(np.float32(c.h))
        a1 = 10.0 / (math.pi * 7.0) if k["data2d"] else 1.0 / math.pi
        a2 = a1 / h ** (2 if k["data2d"] else 3)
        aa = a1 / h ** (3 if k["data2d"] else 4)
        dlt = 1.0 / 1.5
        wdp = a2 * (1.0 - 1.5 * dlt * dlt + 0.75 * dlt ** 3)
        assert k["kernel"] == 1
        for key, v in (("cub_a2", a2), ("cub_a24", 0.25 * a2), ("cub_c1", -3 * aa), ("cub_d1", 9 * aa / 4),
                       ("cub_c2", -3 * aa / 4), ("cub_od_wdeltap", 1 / wdp)):
            assert k[key] == pytest.approx(v, rel=1e-6), key
        assert k["kernelsize"] == pytest.approx(2 * h, rel=1e-7)
