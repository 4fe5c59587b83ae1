"""ctypes binding of libeggroll.so — the C-ABI declared in include/eggroll.h.

The product path has NO CPU / PyTorch fallback: if the HIP library is missing or a call
fails, an exception is raised.  Build it with `python -m hyperscalees_t2i_amd.build_ext`.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import re
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "_build" / "libeggroll.so"
HEADER = _PKG.parent / "include" / "eggroll.h"
SOURCE_FILES = [_PKG / "csrc" / n for n in ("eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip", "common.h")] \
    + [HEADER]

i32, i64, u32, u64, f32 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
vp = C.c_void_p

# name -> (restype, argtypes); mirrors include/eggroll.h exactly (checked by tests)
SIGNATURES = {
    "eggroll_version": (C.c_char_p, []),
    "eggroll_last_error": (C.c_char_p, []),
    "eggroll_noise_factors": (C.c_int, [u64, i64, i64, i64, i64, vp, vp]),
    "eggroll_philox_words": (C.c_int, [u64, i64, i64, vp, vp]),
    "eggroll_perturb": (C.c_int, [vp, vp, i64, i64, vp, vp, i64, i64, i32, i32, i32, i64, i64, f32, vp, i64, vp]),
    "eggroll_perturb_seeded": (C.c_int, [u64, vp, vp, vp, i64, i64, i32, i32, i32, i64, i64, f32, vp, i64, vp]),
    "eggroll_tile_table": (i64, [vp, i32, i32, vp, i64]),
    "eggroll_fitness": (C.c_int, [vp, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp, vp]),
    "eggroll_update_workspace_bytes": (i64, [i64]),
    "eggroll_update": (C.c_int, [vp, vp, i64, i64, vp, vp, i32, i32, vp, vp, i64, i64, i32, f32, f32, f32, vp, vp,
                                 vp]),
    "eggroll_update_seeded": (C.c_int, [u64, vp, vp, vp, i32, i32, vp, vp, i64, i64, i32, f32, f32, f32, vp, vp, vp]),
    "eggroll_lora_linear_pop": (C.c_int, [vp, i64, vp, i64, vp, vp, i64, i64, i64, i32, f32, i64, i64, i64, i64, vp,
                                          i64, vp, vp]),
    "eggroll_lora_gemm": (C.c_int, [vp, i64, vp, i64, vp, vp, vp, i64, i64, i32, f32, i64, i64, i64, i64, vp, i64, vp]),
    "eggroll_lora_gemm_sel": (C.c_int, [vp, i64, vp, i64, vp, vp, vp, i64, i64, i32, f32, i64, i64, i64, i64, vp, i64,
                                        i32, vp]),
    "eggroll_lora_linear_pop_sel": (C.c_int, [vp, i64, vp, i64, vp, vp, i64, i64, i64, i32, f32, i64, i64, i64, i64,
                                              vp, i64, vp, i32, vp]),
    "eggroll_lora_workspace_bytes": (i64, [i64, i64, i32, i64]),
    "eggroll_lora_project": (C.c_int, [vp, i64, vp, i64, i64, i32, i64, i64, i64, vp, vp]),
    "eggroll_lora_project_multi": (C.c_int, [vp, i64, vp, i64, vp, i32, i32, i64, i64, i64, vp, vp]),
    "eggroll_lora_delta_f32": (C.c_int, [vp, i64, vp, i64, vp, i64, i32, f32, i64, i64, i64, i64, vp, i64, vp]),
    "eggroll_dwconv_nhwc": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i32, i32, i32, vp, vp]),
    "eggroll_rownorm": (C.c_int, [vp, i64, i64, f32, i32, vp, vp, vp, vp, i64, i64, i32, vp, vp, vp]),
    "eggroll_gated_residual": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, vp]),
    "eggroll_rownorm_ex": (C.c_int, [vp, i32, i64, i64, f32, i32, vp, vp, vp, vp, i64, i32, i64, i32, vp, i32, vp, i32,
                                     vp, vp]),
    "eggroll_subpixel_shortcut_f32": (C.c_int, [vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, vp]),
    "eggroll_gated_residual_f32": (C.c_int, [vp, vp, vp, i32, i64, i64, i64, i64, vp, vp]),
    "eggroll_resid_layernorm": (C.c_int, [vp, i64, vp, i64, i64, i64, f32, vp, vp, vp, vp]),
    "eggroll_dwconv_pw_nhwc": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i32, vp, vp]),
    "eggroll_dwconv_nhwc_sel": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i32, i32, i32, vp, i32, vp]),
    "eggroll_qk_norm_rope": (C.c_int, [vp, i64, i64, i32, i32, f32, vp, vp, vp, i64, vp]),
    "eggroll_qk_norm_rope_kv": (C.c_int, [vp, i64, i64, i32, i32, f32, vp, vp, vp, i64, vp, vp, i64, i64, i64, i64, vp, i64, vp, vp]),
    "eggroll_group_norm_workspace_bytes": (C.c_int64, [i64, i64, i32, i32]),
    "eggroll_group_norm_nhwc": (C.c_int, [vp, i64, i64, i32, i32, f32, vp, vp, i32, vp, vp, vp]),
    "eggroll_flash_attention": (C.c_int, [vp, i64, i64, vp, i64, i64, vp, i64, i64, i64, i64, i64, i64, i64, f32, vp, i64, i64, vp]),
    "eggroll_flash_attention_sel": (C.c_int, [vp, i64, i64, vp, i64, i64, vp, i64, i64, i64, i64, i64, i64, i64, f32, vp, i64, i64, i32, vp]),
    "eggroll_dwconv_nhwc_ex": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i32, i32, i32, vp, i64, i32, vp]),
    "eggroll_dwconv_pw_nhwc_sel": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i32, vp, i32, vp]),
    "eggroll_upshortcut_add": (C.c_int, [vp, vp, i64, i64, i64, i64, i64, vp]),
    "eggroll_subpixel_shortcut": (C.c_int, [vp, vp, vp, vp, i64, i64, i64, i64, i64, vp]),
    "eggroll_bias_act": (C.c_int, [vp, vp, i64, i64, i32, vp]),
    "eggroll_conv3x3_nhwc": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, i32, vp, vp]),
    "eggroll_conv_nhwc": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, i32, i32, vp, vp]),
    "eggroll_conv3x3_rmsnorm_nhwc": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, C.c_float, vp, vp, vp, vp,
                                               vp]),
    "eggroll_conv_nhwc_sel": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, i32, i32, vp, i32, vp]),
    "eggroll_conv2x2_subpixel_nhwc": (C.c_int, [vp, vp, vp, vp, i32, i64, i64, i64, i64, i64, vp, vp, vp]),
    "eggroll_conv3x3_rmsnorm_nhwc_sel": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, C.c_float, vp, vp, vp,
                                                   vp, i32, vp]),
    "eggroll_dcae_head": (C.c_int, [vp, i64, i64, i64, i64, f32, vp, vp, vp, vp, vp, vp]),
    "eggroll_linear_attention_workspace_bytes": (i64, [i64, i64, i64]),
    "eggroll_linear_attention": (C.c_int, [vp, vp, vp, i64, i64, i64, i64, i64, i32, vp, i64, vp, vp]),
    "eggroll_lora_expand": (C.c_int, [vp, vp, i64, i64, i32, f32, i64, i64, i64, vp, i64, vp]),
    "eggroll_lora_linear_pop_epi": (C.c_int, [vp, i64, vp, i64, vp, vp, i64, i64, i64, i32, f32, i64, i64, i64, i64,
                                              vp, i64, vp, i32, vp, i64, vp, i64, i64, vp]),
    "eggroll_lora_linear_pop_epi_sel": (C.c_int, [vp, i64, vp, i64, vp, vp, i64, i64, i64, i32, f32, i64, i64, i64,
                                                  i64, vp, i64, vp, i32, vp, i64, vp, i64, i64, i32, vp]),
    "eggroll_lora_gemm_epi_sel": (C.c_int, [vp, i64, vp, i64, vp, vp, vp, i64, i64, i32, f32, i64, i64, i64, i64,
                                            vp, i64, i32, vp, i64, vp, i64, i64, i32, vp]),
    "eggroll_cross_attention": (C.c_int, [vp, i64, vp, vp, i64, vp, vp, i64, i64, i64, i64, i64, i64, f32, vp, i64,
                                         vp]),
    "eggroll_cross_attention_sel": (C.c_int, [vp, i64, vp, vp, i64, vp, vp, i64, i64, i64, i64, i64, i64, f32, vp,
                                             i64, i32, vp]),
    "eggroll_clip_preprocess": (C.c_int, [vp, i64, i64, i64, i64, i64, i64, i64, i32, vp, vp, i32, i32, i64, i64,
                                          i64, vp, vp, vp, vp, vp]),
}

_lib = None


class EggrollError(RuntimeError):
    pass


def header_symbols() -> list:
    """Function names declared in include/eggroll.h."""
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"\b(eggroll_[a-z0-9_]+)\s*\(", txt)))


def source_digest() -> str:
    """sha256 over the library's sources + public header (what build_ext compiles)."""
    h = hashlib.sha256()
    for f in SOURCE_FILES:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def check_fresh(path: Path = LIB_PATH) -> None:
    """Raise if the library at `path` was not built from the sources in this tree.

    build_ext writes the digest of the sources it compiled next to the library; a prebuilt .so
    pushed with a newer source tree (or an older one) is refused instead of silently tested."""
    stamp = path.with_name(path.name + ".srcsha256")
    if not all(f.exists() for f in SOURCE_FILES):
        return  # installed without sources: nothing to compare against
    if not stamp.exists():
        raise EggrollError(f"{path} has no source stamp ({stamp.name}): rebuild with "
                           "`python -m hyperscalees_t2i_amd.build_ext --force`")
    if stamp.read_text().strip() != source_digest():
        raise EggrollError(f"stale {path}: csrc/ or include/eggroll.h changed since it was built; rebuild with "
                           "`python -m hyperscalees_t2i_amd.build_ext`")


def load():
    global _lib
    if _lib is not None:
        return _lib
    override = os.environ.get("EGGROLL_LIB")
    path = Path(override or LIB_PATH)
    if not path.exists():
        raise EggrollError(
            f"libeggroll.so not found at {path}: build it with `python -m hyperscalees_t2i_amd.build_ext` "
            "(there is no CPU fallback)")
    if not override:
        check_fresh(path)
    lib = C.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().eggroll_last_error().decode(errors="replace")
        raise EggrollError(f"{what} failed (rc={rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def version() -> str:
    return load().eggroll_version().decode()
