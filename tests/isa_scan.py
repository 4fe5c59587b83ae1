"""ISA scan for the round-3 fault class: a scalar load through a DATA pointer issued
inside a divergent block that no `s_cbranch_execz` guards.

Scalar loads ignore EXEC, so such a load executes on every wave even when no lane takes the branch.
If its address is only in bounds when the branch is taken (k_update's fit[2h] at even pop), the wave
reads past the buffer and faults whenever that buffer ends a mapped segment.  Kernel-argument loads
(through the kernarg segment pointer, always mapped) are harmless and not reported.

Method (linear, per function, conservative for this code base): after an instruction that narrows
EXEC (s_and_saveexec / s_andn2_saveexec / s_and_b64 exec / s_andn2_b64 exec / s_xor_b64 exec) the
block is "unguarded" until an `s_cbranch_execz` (the fall-through then has live lanes) or an
`s_or_b64 exec` join; a scalar load there whose base register pair is not the function's kernarg
pointer (the base of the function's first scalar load) is reported.  Uses the ROCm LLVM tools
(llvm-objcopy, clang-offload-bundler, llvm-objdump) on the built objects; no GPU.
"""
from __future__ import annotations

import re
import subprocess
import tempfile
from pathlib import Path
from typing import List, Tuple

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_NARROW = re.compile(r"^\s*(s_and_saveexec_b64|s_andn2_saveexec_b64|s_and_b64 exec,|s_andn2_b64 exec,|s_xor_b64 exec,)")
_JOIN = re.compile(r"^\s*s_or_b64 exec,")
_GUARD = re.compile(r"^\s*s_cbranch_execz")
_SLOAD = re.compile(r"^\s*(s_load_\w+|s_buffer_load_\w+)\s+[^,]+,\s*(s\[\d+:\d+\])")


def tools_present() -> bool:
    return all((LLVM / t).exists() for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"))


def disassemble(obj: Path) -> str:
    """Device ISA of one hipcc-built host object (its .hip_fatbin bundle, gfx950 entry)."""
    with tempfile.TemporaryDirectory() as td:
        fb, co = Path(td) / "fb.bin", Path(td) / "dev.co"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(obj)], check=True,
                       capture_output=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", f"--input={fb}", f"--targets={TARGET}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                              capture_output=True, text=True).stdout


def scan(isa: str) -> List[Tuple[str, str]]:
    """[(function, instruction)] of scalar data-pointer loads in unguarded divergent blocks."""
    hits: List[Tuple[str, str]] = []
    fn, karg, unguarded = "?", None, False
    for line in isa.splitlines():
        m = _FUNC.match(line.strip())
        if m:
            fn, karg, unguarded = m.group(1), None, False
            continue
        ins = line.split("//")[0]
        if _NARROW.match(ins):
            unguarded = True
        elif _GUARD.match(ins) or _JOIN.match(ins):
            unguarded = False
        m = _SLOAD.match(ins)
        if m:
            if karg is None:
                karg = m.group(2)
            elif unguarded and m.group(2) != karg:
                hits.append((fn, ins.strip()))
    return hits
