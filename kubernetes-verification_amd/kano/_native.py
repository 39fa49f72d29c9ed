"""ctypes binding of libkano_hip.so (C ABI: include/kano_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc,
--offload-arch=gfx950) into ``kubernetes-verification_amd/csrc/``.  There is
no CPU fallback: every compute entry point of the drop-in API goes through
this library and raises ``KanoNativeError`` when it is missing or when no GPU
is visible.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_uint8, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "KANO_HIP_LIB", os.path.join(os.path.dirname(_HERE), "csrc", "libkano_hip.so"))

# Exported symbols, exactly the declarations of include/kano_hip.h.
SIGNATURES = {
    "kano_create": (c_int, [c_int, POINTER(c_void_p)]),
    "kano_create_lean": (c_int, [c_int, POINTER(c_void_p)]),
    "kano_destroy": (None, [c_void_p]),
    "kano_last_error": (ctypes.c_char_p, [c_void_p]),
    "kano_set_stream": (c_int, [c_void_p, c_void_p]),
    "kano_set_pods": (c_int, [c_void_p, c_int64, c_int32, c_void_p]),
    "kano_set_policies": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "kano_set_shard": (c_int, [c_void_p, c_int64, c_int64]),
    "kano_build": (c_int, [c_void_p, c_int]),
    "kano_info": (c_int, [c_void_p, c_void_p]),
    "kano_col_checks": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kano_col_flags_dev": (c_int, [c_void_p, c_void_p]),
    "kano_crosscheck": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kano_crosscheck_dev": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kano_get_rows": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "kano_rows_digest": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "kano_checks_shard": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_void_p]),
    "kano_put_rows": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "kano_get_col": (c_int, [c_void_p, c_int64, c_void_p]),
    "kano_get_bit": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_int)]),
    "kano_set_bit": (c_int, [c_void_p, c_int64, c_int64, c_int]),
    "kano_get_policy_sets": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "kano_get_classes": (c_int, [c_void_p, c_void_p]),
    "kano_get_select_csr": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kano_get_allow_csr": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kano_shadow": (c_int, [c_void_p, POINTER(c_int64)]),
    "kano_shadow_fetch": (c_int, [c_void_p, c_void_p]),
    "kano_shadow_lists": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                  c_void_p, POINTER(c_int64)]),
    "kano_conflict": (c_int, [c_void_p, POINTER(c_int)]),
    "kano_verify": (c_int, [c_void_p, c_int, c_void_p, c_int32, c_int64, c_void_p, c_void_p,
                            c_void_p, c_int64, POINTER(c_int64)]),
    "kano_verify_shard": (c_int, [c_void_p, c_int, c_void_p, c_int32, c_int64, c_int, c_void_p]),
    "kano_verify_combine": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                    c_int64, POINTER(c_int64)]),
    "kano_verify_gather": (c_int, [c_void_p, c_int, c_void_p, c_int32, c_int64, c_int, c_void_p,
                                   c_int32, c_void_p, c_void_p, c_void_p, c_int64,
                                   POINTER(c_int64)]),
    "kano_set_groups": (c_int, [c_void_p, c_void_p, c_int32]),
    "kano_set_expressions": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kano_path": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "kano_k8s_edge": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "kano_build_classes": (c_int, [c_void_p, c_int]),
    "kano_path_shard_words": (c_int, [c_void_p, POINTER(c_int64)]),
    "kano_path_shard": (c_int, [c_void_p, c_void_p]),
    "kano_path_combine": (c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_int, c_int,
                                  c_void_p]),
    "kano_export_rows": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "kano_add_policies": (c_int, [c_void_p, c_int64, c_int32, c_void_p] + [c_void_p] * 6 +
                          [POINTER(c_int64)]),
    "kano_remove_policies": (c_int, [c_void_p, c_int64, c_void_p]),
    "kano_added_policy_sets": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "kano_import_rows": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "kano_stage_times": (c_int, [c_void_p, c_void_p]),
    "kano_rows_timing": (c_int, [c_void_p, c_void_p, c_int]),
    "kano_host_times": (c_int, [c_void_p, c_void_p, c_int]),
    "kano_set_pipeline": (c_int, [c_void_p, c_int]),
    "kano_settle": (c_int, [c_void_p]),
    "kano_gate_timing": (c_int, [c_void_p, c_int, POINTER(c_int64), POINTER(c_double),
                                 POINTER(c_double)]),
    "kano_mfma_timing": (c_int, [c_void_p, c_void_p, c_int]),
    "kano_group_create": (c_int, [c_int, c_void_p, POINTER(c_void_p)]),
    "kano_group_create_lean": (c_int, [c_int, c_void_p, POINTER(c_void_p)]),
    "kano_group_create_ex": (c_int, [c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "kano_group_destroy": (None, [c_void_p]),
    "kano_group_last_error": (ctypes.c_char_p, [c_void_p]),
    "kano_group_info": (c_int, [c_void_p, c_void_p]),
    "kano_group_member": (c_int, [c_void_p, c_int, POINTER(c_void_p)]),
    "kano_group_verify": (c_int, [c_void_p, c_int, c_void_p, c_int32, c_int64, c_int, c_void_p,
                                  c_void_p, c_void_p, c_int64, POINTER(c_int64)]),
    "kano_group_checks": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p]),
    "kano_group_upload": (c_int, [c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kano_group_build": (c_int, [c_void_p, c_int]),
    "kano_group_set_groups": (c_int, [c_void_p, c_void_p, c_int32]),
    "kano_group_add_policies": (c_int, [c_void_p, c_int64, c_int32, c_void_p] + [c_void_p] * 6 +
                                [POINTER(c_int64)]),
    "kano_group_remove_policies": (c_int, [c_void_p, c_int64, c_void_p]),
    "kano_group_path": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "kano_group_exchange_timing": (c_int, [c_void_p, c_int, c_void_p, c_int]),
    "kano_host_alloc": (c_int, [ctypes.c_size_t, POINTER(c_void_p)]),
    "kano_host_free": (None, [c_void_p]),
}

INFO_SLOTS = 17
INFO = dict(N=0, W=1, P=2, U=3, NNZ_SEL=4, NNZ_ALW=5, HEAVY=6, ROW0=7, ROW1=8, MAXSEL=9,
            UA=10, HEAVY_PATH=11, WORK_ITEMS=12, ROWS_KERNEL=13, ROWS_CUS=14,
            HEAVY_SEL=15, HEAVY_KERNEL=16)
PATHS = {"auto": 0, "bitwise": 1, "mfma": 2}
STORED_GROUPS = -1   # KANO_STORED_GROUPS
GROUP_LEAN, GROUP_RCCL, GROUP_COPY = 1, 2, 4   # KANO_GROUP_* flags


class KanoNativeError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libkano_hip.so and attach the C signatures (no GPU needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KanoNativeError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(ctx, rc: int, what: str) -> None:
    if rc != 0:
        msg = ""
        if ctx:
            raw = load().kano_last_error(ctx)
            msg = raw.decode(errors="replace") if raw else ""
        raise KanoNativeError(f"{what} failed (rc={rc}): {msg}")


def gpu_available() -> bool:
    """True when the library loads and a HIP device can be opened."""
    try:
        lib = load()
    except (KanoNativeError, OSError):
        return False
    ctx = c_void_p()
    rc = lib.kano_create(0, ctypes.byref(ctx))
    if rc == 0:
        lib.kano_destroy(ctx)
        return True
    return False
