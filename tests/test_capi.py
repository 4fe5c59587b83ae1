"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/eggroll.h declares, and rejects bad arguments with a message (no kernel launched)."""
import ctypes as C
import subprocess

import numpy as np
import pytest

from hyperscalees_t2i_amd import _lib
from hyperscalees_t2i_amd.kernels import ThetaLayout
from oracle import eggroll_oracle as O


def test_library_loads_and_versions():
    lib = _lib.load()
    assert _lib.version().startswith("eggroll-mi355x")
    assert lib.eggroll_last_error() is not None


def test_exports_match_header():
    declared = _lib.header_symbols()
    assert set(declared) == set(_lib.SIGNATURES), "ctypes signatures drift from include/eggroll.h"
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("eggroll_")}
    assert exported == set(declared)


def test_header_compiles_as_c():
    src = '#include "eggroll.h"\nint main(void){eggroll_mat_t m; (void)m; return (int)sizeof(eggroll_mat_t) - 48;}\n'
    r = subprocess.run(["gcc", "-x", "c", "-std=c99", "-Wall", "-Werror", f"-I{_lib.HEADER.parent}", "-", "-o",
                        "/tmp/eggroll_hdr_test"], input=src, text=True, capture_output=True)
    assert r.returncode == 0, r.stderr
    assert subprocess.run(["/tmp/eggroll_hdr_test"]).returncode == 0


def test_argument_errors_are_reported():
    lib = _lib.load()
    rc = lib.eggroll_fitness(None, 0, 4, 1, 1e-8, None, None, None, None, None, None, None)
    assert rc == -1 and b"fitness" in lib.eggroll_last_error()
    rc = lib.eggroll_noise_factors(0, 0, 2, 10, 9, None, None)  # ld not multiple of 4
    assert rc == -1 and b"ld" in lib.eggroll_last_error()
    rc = lib.eggroll_lora_linear_pop(None, 64, None, 64, None, None, 0, 0, 0, 2, 1.0, 10, 10, 10, 60, None, 10,
                                     None, None)  # K % 64 != 0
    assert rc == -1 and b"multiple of 64" in lib.eggroll_last_error()
    rc = lib.eggroll_lora_linear_pop_sel(None, 64, None, 64, None, None, 0, 0, 0, 2, 1.0, 10, 10, 10, 64, None, 10,
                                         None, 11, None)  # kernel 11: not a kernel id
    assert rc == -1 and b"kernel" in lib.eggroll_last_error()
    rc = lib.eggroll_lora_gemm_sel(None, 64, None, 64, None, None, None, 0, 0, 2, 1.0, 10, 10, 10, 64, None, 10, 12,
                                   None)  # kernel 12 (fused projection) exists only in linear_pop_sel
    assert rc == -1 and b"12" in lib.eggroll_last_error()
    with pytest.raises(_lib.EggrollError):
        _lib.check(-1, "probe")


def test_zero_sized_calls_are_noops():
    lib = _lib.load()
    assert lib.eggroll_noise_factors(0, 3, 3, 16, 16, None, None) == 0
    assert lib.eggroll_lora_project(None, 64, None, 64, 0, 2, 4, 0, 64, None, None) == 0


def test_layout_matches_oracle():
    shapes = [(2, 2240), (2240, 2), (6,), (2, 256), (13440, 2)]
    for r in (1, 2, 4):
        a = ThetaLayout(shapes, r)
        b = O.layout(shapes, r)
        assert np.array_equal(a.mats, b["mats"]) and a.D == b["D"] and a.factor_len == b["factor_len"]
        assert a.total_chunks == b["total_chunks"] and a.factor_ld % 4 == 0


def _tile_kind(m, n, toff, foff, r):
    """include/eggroll.h tile rule restated (common.h egg_tile_kind)."""
    al = toff % 4 == 0 and foff % 4 == 0
    if n == 0:
        return "vec4" if (al and m % 4 == 0) else "vec"
    rok = r in (1, 2, 4)
    if rok and al and m <= n and m in (1, 2, 4) and n % 4 == 0:
        return "wide"
    if rok and al and n < m and n in (1, 2, 4) and m % 4 == 0:
        return "tall"
    return "gen"


def test_tile_table_covers_every_matrix():
    shapes = [(2, 2240), (2240, 2), (6,), (7,), (2, 256), (13440, 2), (3, 5), (4, 12), (12, 4), (1, 1), (2, 30)]
    for r in (1, 2, 3, 4):
        lay = ThetaLayout(shapes, r)
        t = lay.tile_table()
        assert t.dtype == np.int32 and t.shape[1] == 2
        want = []
        for i, (m, n, toff, foff, _, _) in enumerate(lay.mats.tolist()):
            k = _tile_kind(m, n, toff, foff, r)
            long = {"wide": n, "tall": m, "vec4": m, "vec": m, "gen": m * n}[k]
            want += [(i, j) for j in range(-(-long // 1024))]
        assert [tuple(x) for x in t.tolist()] == want, r
        assert all(f % 4 == 0 for f in lay.mats[:, 3])            # every factor segment 16-byte aligned


def test_factor_pack_roundtrip():
    shapes = [(2, 7), (5, 2), (3,), (1, 1)]
    lay = ThetaLayout(shapes, 2)
    x = np.arange(3 * lay.factor_len_packed, dtype=np.float32).reshape(3, -1)
    p = lay.pack_factors(x)
    assert p.shape == (3, lay.factor_ld) and np.array_equal(lay.unpack_factors(p), x)
    assert lay.factor_len_packed == 2 * (2 + 7) + 2 * (5 + 2) + 3 + 2 * 2


# --------------------------------------------------------------------------------------------
# The documented binding == _lib.SIGNATURES == the header's prototypes
# --------------------------------------------------------------------------------------------
import re  # noqa: E402
from pathlib import Path  # noqa: E402

_CT = {"vp": C.c_void_p, "i32": C.c_int32, "i64": C.c_int64, "u32": C.c_uint32, "u64": C.c_uint64,
       "f32": C.c_float, "C.c_char_p": C.c_char_p}


def _norm(t):
    """ctypes type -> comparable token (c_int is c_int32 on this ABI)."""
    return {C.c_int: "i32", C.c_int32: "i32", C.c_int64: "i64", C.c_uint32: "u32", C.c_uint64: "u64",
            C.c_float: "f32", C.c_void_p: "vp", C.c_char_p: "str"}[t]


def header_prototypes():
    """{name: (ret, [arg tokens])} parsed from include/eggroll.h (pointers -> vp)."""
    txt = re.sub(r"/\*.*?\*/", "", _lib.HEADER.read_text(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"(const char\s*\*|int64_t|int)\s+(eggroll_\w+)\s*\(([^;]*?)\)\s*;", txt):
        toks = []
        for a in [a.strip() for a in args.split(",") if a.strip() and a.strip() != "void"]:
            if "*" in a:
                toks.append("vp")
            else:
                base = a.replace("const ", "").split()[0]
                toks.append({"int64_t": "i64", "int32_t": "i32", "uint64_t": "u64", "uint32_t": "u32",
                             "float": "f32", "int": "i32"}[base])
        out[name] = ({"int": "i32", "int64_t": "i64"}.get(ret, "str"), toks)
    return out


def integration_blocks():
    md = (Path(__file__).resolve().parent.parent / "INTEGRATION.md").read_text()
    return re.findall(r"```python\n(.*?)```", md, flags=re.S)


def test_signatures_match_header_prototypes():
    proto = header_prototypes()
    assert set(proto) == set(_lib.SIGNATURES)
    for name, (res, args) in _lib.SIGNATURES.items():
        assert proto[name] == (_norm(res), [_norm(a) for a in args]), name


def test_integration_stub_matches_header():
    stub = integration_blocks()[0]
    got = {}
    for name, res, args in re.findall(r"lib\.(eggroll_\w+)\.restype, lib\.\1\.argtypes = ([\w.]+), \[([^\]]*)\]", stub):
        got[name] = (_norm(_CT[res]), [_norm(_CT[a.strip()]) for a in args.split(",") if a.strip()])
    assert set(got) == set(_lib.SIGNATURES), "INTEGRATION.md stub drifts from the library's exports"
    for name, (res, args) in _lib.SIGNATURES.items():
        assert got[name] == (_norm(res), [_norm(a) for a in args]), name


def test_integration_stub_binds_the_library():
    """The stub's bind() runs against the built library, and its theta_records / tile_table helpers
    reproduce the package's own layout and tile table."""
    ns = {}
    exec(integration_blocks()[0], ns)
    lib = ns["bind"](str(_lib.LIB_PATH))
    assert lib.eggroll_version().decode().startswith("eggroll-mi355x")
    shapes = [(2, 2240), (2240, 2), (6,), (2, 30), (13440, 2), (3, 5)]
    for r in (1, 2, 4):
        mats, D, flen = ns["theta_records"](shapes, r)
        lay = ThetaLayout(shapes, r)
        assert np.array_equal(mats, lay.mats) and D == lay.D and flen == lay.factor_len
        assert np.array_equal(ns["tile_table"](lib, mats, r), lay.tile_table())


def test_tile_table_rejects_oversized_generic_matrix():
    """The generic per-element path indexes in 32-bit ints: a T_GEN matrix of >= 2^31 elements is an
    argument error, not a silent overflow (fast-path tiles have no such limit)."""
    lib = _lib.load()
    big = np.array([[3, 1 << 30, 0, 0, 0, 0]], dtype=np.int64)        # rank 3: generic tiles, 3 * 2^30 elements
    assert lib.eggroll_tile_table(big.ctypes.data, 1, 3, None, 0) == -1
    assert b"too large" in lib.eggroll_last_error()
    ok = np.array([[2, 1 << 30, 0, 0, 0, 0]], dtype=np.int64)         # lora_A-shaped, rank 1: wide tiles
    assert lib.eggroll_tile_table(ok.ctypes.data, 1, 1, None, 0) == (1 << 30) // 1024


def test_stale_library_is_refused(tmp_path):
    """_lib.check_fresh: a library whose source stamp is missing or differs from today's sources is
    refused (what conftest and _lib.load() run before any test touches it)."""
    import shutil
    lib = tmp_path / "libeggroll.so"
    shutil.copy(_lib.LIB_PATH, lib)
    with pytest.raises(_lib.EggrollError, match="no source stamp"):
        _lib.check_fresh(lib)
    (tmp_path / "libeggroll.so.srcsha256").write_text("0" * 64 + "\n")
    with pytest.raises(_lib.EggrollError, match="stale"):
        _lib.check_fresh(lib)
    (tmp_path / "libeggroll.so.srcsha256").write_text(_lib.source_digest() + "\n")
    _lib.check_fresh(lib)
    _lib.check_fresh()                       # the in-tree library is current
