"""The round-3 fault class, checked on every build (CPU, no GPU): no scalar load through a data
pointer inside an unguarded divergent block (tests/isa_scan.py).

The one known site is k_update's antithetic collapse `c_j = j < h ? f_j - f_{j+h} : f_{2h}`: the
else-branch fitness read is issued as a scalar load inside the divergent block (it executes even when
no lane takes the branch), and since round 3 its index is clamped into [0, pop) so it is in bounds by
construction (cbe1ac4; `test_update_fitness_vector_at_allocation_end` runs it on the GPU with the
fitness vector at the end of its allocation).  It is allowed here once per k_update instantiation;
any other hit fails the build check and must be read in the ISA before it is allowed.
"""
import re
from pathlib import Path

import pytest

import isa_scan

BUILD = Path(__file__).resolve().parent.parent / "hyperscalees_t2i_amd" / "_build"
ALLOWED = re.compile(r"^_ZN7eggroll8k_update")


@pytest.mark.skipif(not isa_scan.tools_present(), reason="ROCm LLVM tools absent")
@pytest.mark.parametrize("unit", ["eggroll_es", "eggroll_lora", "eggroll_model"])
def test_no_unguarded_scalar_data_loads(unit):
    obj = BUILD / f"{unit}.o"
    if not obj.exists():
        pytest.skip(f"{obj} not built")
    hits = isa_scan.scan(isa_scan.disassemble(obj))
    per_fn = {}
    for fn, ins in hits:
        per_fn.setdefault(fn, []).append(ins)
    bad = {fn: ins for fn, ins in per_fn.items() if not ALLOWED.match(fn) or len(ins) > 1}
    assert not bad, f"scalar data loads in unguarded divergent blocks: {bad}"


def test_scanner_flags_the_pattern():
    """The scanner itself on a hand-written fragment: the kernarg load passes, the data-pointer load
    after s_and_saveexec is flagged, the one behind s_cbranch_execz is not."""
    isa = "\n".join([
        "0000000000001000 <k>:",
        "\ts_load_dwordx4 s[4:7], s[0:1], 0x0",
        "\ts_and_saveexec_b64 s[8:9], vcc",
        "\ts_load_dword s10, s[4:5], 0x0",
        "\ts_load_dword s11, s[0:1], 0x10",
        "\ts_or_b64 exec, exec, s[8:9]",
        "\ts_and_saveexec_b64 s[8:9], vcc",
        "\ts_cbranch_execz 4",
        "\ts_load_dword s12, s[4:5], 0x4",
    ])
    assert isa_scan.scan(isa) == [("k", "s_load_dword s10, s[4:5], 0x0")]
