"""ctypes binding of the C-ABI library libgsplat_mi355x.so (include/gsplat_mi355x.h).

The library is the only compute path: there is no CPU or eager-PyTorch fallback.  If it
is missing, or a tensor is not on a ROCm device, calls raise instead of silently running
something else.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import subprocess

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSPLAT_MI355X_LIB") or os.path.join(_HERE, "libgsplat_mi355x.so")
# the test library (the same sources built with the gsplat_debug_* switches: hooks())
HOOKS_PATH = os.environ.get("GSPLAT_MI355X_HOOKS_LIB") or \
    os.path.join(_HERE, "libgsplat_mi355x_hooks.so")
# measurement switches for A/B runs of bench.py / tools (applied at load): they exist in the
# test library only, so setting one loads that library in place of the shipped one
_SWITCH_ENV = ("GSPLAT_MI355X_RASTER_VARIANT", "GSPLAT_MI355X_CHUNK",
               "GSPLAT_MI355X_DEPTH_KEY_RANGE")
if any(os.environ.get(k) for k in _SWITCH_ENV) and not os.environ.get("GSPLAT_MI355X_LIB"):
    LIB_PATH = HOOKS_PATH
CSRC = os.path.join(_HERE, "csrc")

_c = ctypes
_P = _c.c_void_p
_F = _c.c_float
_I = _c.c_int
_I64 = _c.c_int64
_SZ = _c.c_size_t

# name -> (restype, argtypes); must match include/gsplat_mi355x.h exactly.
SIGNATURES = {
    "gsplat_abi_version": (_I, []),
    "gsplat_set_quirks": (_I, [_I]),
    "gsplat_get_quirks": (_I, []),
    "gsplat_set_deterministic": (_I, [_I]),
    "gsplat_get_deterministic": (_I, []),
    "gsplat_last_error": (_c.c_char_p, []),
    "gsplat_project_gaussians_forward": (_I, [
        _I, _P, _P, _F, _P, _P, _P, _F, _F, _F, _F, _I, _I, _I, _I, _F,
        _P, _P, _P, _P, _P, _P, _P]),
    "gsplat_project_gaussians_forward_binned": (_I, [
        _I, _P, _P, _F, _P, _P, _P, _F, _F, _F, _F, _I, _I, _I, _I, _F,
        _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "gsplat_project_gaussians_backward": (_I, [
        _I, _P, _P, _F, _P, _P, _P, _F, _F, _F, _F, _I, _I, _P, _P, _P, _P, _P, _P,
        _P, _P, _P, _P, _P, _P]),
    "gsplat_compute_sh_forward": (_I, [_I, _I, _I, _P, _P, _P, _P]),
    "gsplat_compute_sh_backward": (_I, [_I, _I, _I, _P, _P, _P, _P]),
    "gsplat_compute_sh_backward_split": (_I, [_I, _I, _I, _P, _P, _P, _P, _P]),
    "gsplat_compute_sh_backward_views": (_I, [_I, _I, _I, _I, _P, _P, _I64, _P, _P]),
    "gsplat_compute_sh_backward_views_split": (_I, [_I, _I, _I, _I, _P, _P, _I64, _P, _P, _P]),
    "gsplat_compute_cov2d_bounds": (_I, [_I, _P, _P, _P, _P]),
    "gsplat_map_gaussian_to_intersects": (_I, [_I, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "gsplat_sort_isect_pairs_workspace_size": (_SZ, [_I64]),
    "gsplat_sort_isect_pairs": (_I, [_I64, _I, _P, _P, _P, _P, _P, _SZ, _P]),
    "gsplat_get_tile_bin_edges": (_I, [_I64, _P, _P, _I64, _P]),
    "gsplat_bin_count_workspace_size": (_SZ, [_I]),
    "gsplat_bin_emit_workspace_size_for": (_SZ, [_I, _I64, _I, _I]),
    "gsplat_bin_count": (_I, [_I, _P, _P, _P, _P, _I, _I, _P, _P, _SZ, _P]),
    "gsplat_bin_emit": (_I, [_I, _I64, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _P]),
    "gsplat_bin_emit_prelaunch": (_I, [_I, _I64, _I, _I, _P, _P, _SZ, _P, _SZ, _P]),
    "gsplat_bin_emit_finish": (_I, [_I, _I64, _I64, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _P]),
    "gsplat_bin_emit_speculative": (_I, [_I, _I64, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _P]),
    "gsplat_rasterize_forward": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                      _P, _P]),
    "gsplat_rasterize_forward_rgbd": (_I, [_I, _I, _I, _I] + [_P] * 13),
    "gsplat_rasterize_backward_workspace_size": (_SZ, [_I, _I]),
    "gsplat_rasterize_chunk_size": (_I, [_I, _I, _I64]),
    "gsplat_rasterize_split_bytes": (_SZ, [_I, _I, _I64, _I]),
    "gsplat_rasterize_forward_clearing": (_I, [_I, _I, _I, _I] + [_P] * 10 +
                                          [_P, _SZ, _P, _I64, _I, _P, _SZ, _P]),
    "gsplat_rasterize_backward_chunked": (_I, [_I, _I, _I, _I, _I] + [_P] * 11 + [_F] +
                                          [_P] * 4 + [_I64, _I, _P, _SZ, _P, _SZ, _P]),
    "gsplat_debug_pair_count": (_I, [_P]),
    "gsplat_l1_ssim_num_blocks": (_I, [_I, _I]),
    "gsplat_l1_ssim_forward": (_I, [_I, _I, _I, _P, _P, _P, _F, _I, _P, _P, _P, _P]),
    "gsplat_l1_ssim_backward": (_I, [_I, _I, _I, _P, _P, _P, _F, _I, _P, _P, _P, _P]),
    "gsplat_adam_step": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _P]),
    "gsplat_rasterize_backward": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                       _P, _P, _P, _F, _P, _P, _P, _P, _P, _SZ, _P]),
    "gsplat_fused_preprocess_forward": (_I, [_I, _I, _I] + [_P] * 9 + [_F] * 4 +
                                        [_I] * 4 + [_F] + [_P] * 11),
    "gsplat_fused_preprocess_forward_binned": (_I, [_I, _I, _I] + [_P] * 9 + [_F] * 4 +
                                               [_I] * 4 + [_F] + [_P] * 8 + [_SZ, _P]),
    "gsplat_fused_preprocess_forward_part": (_I, [_I, _I, _I, _I] + [_P] * 9 + [_F] * 4 +
                                             [_I] * 4 + [_F] + [_P] * 8 + [_SZ, _P]),
    "gsplat_bin_count_keyed": (_I, [_I, _I, _I, _P, _P, _SZ, _P]),
    "gsplat_bin_count_keyed_ex": (_I, [_I, _I, _I, _P, _P, _SZ, _c.c_uint32, _P]),
    "gsplat_bin_speculative": (_I, [_I, _I64, _I, _I, _P, _P, _SZ, _c.c_uint32, _P, _P, _P, _SZ,
                                    _P]),
    "gsplat_fused_preprocess_backward": (_I, [_I, _I, _I] + [_P] * 6 + [_F] * 4 + [_I, _I] +
                                         [_P] * 13),
    "gsplat_fused_preprocess_backward_adam": (_I, [_I, _I, _I] + [_P] * 9 + [_F] * 4 +
                                              [_I, _I] + [_P] * 8 + [_I, _F, _F, _F, _P]),
    "gsplat_exchange_pack_colors": (_I, [_I, _P, _SZ, _P, _P, _P, _P, _P]),
    "gsplat_exchange_sparse_floats": (_I64, [_I, _I64]),
    "gsplat_exchange_sparse_plan": (_I, [_I, _P, _P, _P]),
    "gsplat_exchange_pack_sparse": (_I, [_I, _P, _SZ, _P, _P, _P, _P, _I64, _P]),
    "gsplat_fused_preprocess_backward_accumulate": (_I, [_I, _I, _I] + [_P] * 6 + [_F] * 4 +
                                                    [_I, _I] + [_P] * 11),
    "gsplat_compute_sh_backward_view_table": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gsplat_compute_sh_backward_view_table_adam": (
        _I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F, _I, _F, _F, _F, _P]),
    "gsplat_grad_records_bytes": (_SZ, [_I]),
    "gsplat_grad_records_split": (_I, [_I, _P, _SZ, _P, _P, _P, _P, _P, _P, _P]),
    "gsplat_rasterize_backward_records": (_I, [_I] * 5 + [_P] * 11 + [_F, _I64, _I, _P, _SZ,
                                                                       _I, _P, _SZ, _P]),
    "gsplat_rasterize_l1_partials_bytes": (_SZ, [_I, _I]),
    "gsplat_rasterize_forward_clearing_l1": (_I, [_I, _I, _I, _I] + [_P] * 10 +
                                             [_P, _SZ, _P, _I64, _I, _P, _SZ] +
                                             [_P, _I, _P, _SZ, _P, _P]),
    "gsplat_rasterize_backward_records_l1": (_I, [_I] * 5 + [_P] * 9 + [_P, _P, _I, _P] +
                                             [_F, _I64, _I, _P, _SZ, _I, _P, _SZ, _P]),
}

# the test library's extra entries (include/gsplat_mi355x.h "test hooks", GSPLAT_TEST_HOOKS)
HOOK_SIGNATURES = {
    "gsplat_debug_binning_scheme": (_I, [_I]),
    "gsplat_debug_set_chunk": (_I, [_I]),
    "gsplat_debug_set_raster_variant": (_I, [_I, _I, _I]),
    "gsplat_debug_raster_variant_is_default": (_I, []),
    "gsplat_debug_depth_key_range": (_I, [_I]),
    "gsplat_debug_wave_log": (_I, [_P]),
    "gsplat_debug_tile_sort_gen": (_I64, [_I64]),
    "gsplat_debug_emit_counts": (_I, [_I]),
}

ABI_VERSION = 17  # include/gsplat_mi355x.h GSPLAT_MI355X_ABI_VERSION

_lib = None
_DETERMINISTIC = os.environ.get("GSPLAT_MI355X_DETERMINISTIC", "0") not in ("", "0")


def set_deterministic(on: bool) -> bool:
    """Deterministic rasterize backward (integer accumulation; bit-identical gradients run to
    run, slower -- a debugging mode).  Also GSPLAT_MI355X_DETERMINISTIC=1.  Returns the previous
    setting."""
    global _DETERMINISTIC
    prev, _DETERMINISTIC = _DETERMINISTIC, bool(on)
    if _lib is not None:
        _lib.gsplat_set_deterministic(int(_DETERMINISTIC))
    return prev


def build(jobs: int = 8) -> str:
    """Compile the HIP sources for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"], check=True)
    return LIB_PATH


def _load(path):
    """Load and bind a build of the library (shipped or test), apply the quirks and the
    deterministic setting."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"gsplat MI355X library not built: {path} is missing "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = ctypes.CDLL(path)
    for table in (SIGNATURES, HOOK_SIGNATURES):
        for name, (res, args) in table.items():
            # (an older build loaded for a same-box A/B run, GSPLAT_MI355X_LIB, may lack a newer
            # entry; the shipped library must have every SIGNATURES one)
            if not hasattr(L, name) and (table is HOOK_SIGNATURES or name.startswith(
                    "gsplat_debug_") or os.environ.get("GSPLAT_MI355X_LIB")):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
    if L.gsplat_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{os.path.basename(path)} ABI version mismatch")
    from . import quirks
    if L.gsplat_set_quirks(quirks.get()) != 0:
        raise RuntimeError(L.gsplat_last_error().decode(errors="replace"))
    L.gsplat_set_deterministic(int(_DETERMINISTIC))
    return L


def lib():
    global _lib
    if _lib is None:
        L = _load(LIB_PATH)
        # measurement switches (A/B runs; LIB_PATH is then the test library):
        # GSPLAT_MI355X_RASTER_VARIANT = "fwd_pxl,bwd_pxl,flags" (gsplat_debug_set_raster_variant;
        # "/" separates as well, for tools/gpu_iter.sh's comma-separated env lists),
        # GSPLAT_MI355X_CHUNK = the list-split chunk override (gsplat_debug_set_chunk)
        var = os.environ.get("GSPLAT_MI355X_RASTER_VARIANT")
        if var and L.gsplat_debug_set_raster_variant(*[int(x) for x in var.replace("/", ",").split(",")]) != 0:
            raise RuntimeError(L.gsplat_last_error().decode(errors="replace"))
        if os.environ.get("GSPLAT_MI355X_CHUNK"):
            L.gsplat_debug_set_chunk(int(os.environ["GSPLAT_MI355X_CHUNK"]))
        if os.environ.get("GSPLAT_MI355X_DEPTH_KEY_RANGE"):  # 0 off, 1 from 2^22 keys, 2 always
            L.gsplat_debug_depth_key_range(int(os.environ["GSPLAT_MI355X_DEPTH_KEY_RANGE"]))
        _lib = L
    return _lib


_hooks_lib = None


@contextlib.contextmanager
def hooks():
    """Run the C ABI through the test library (libgsplat_mi355x_hooks.so: the shipped kernels
    plus the gsplat_debug_* switches) for the duration: tests that select non-default paths.
    Yields that library; the switches must be restored before leaving (each test does)."""
    global _lib, _hooks_lib
    prev = lib()
    if _hooks_lib is None:
        _hooks_lib = _load(HOOKS_PATH)
    from . import quirks
    _hooks_lib.gsplat_set_quirks(quirks.get())
    _hooks_lib.gsplat_set_deterministic(int(_DETERMINISTIC))
    _lib = _hooks_lib
    try:
        yield _hooks_lib
    finally:
        _lib = prev
        # (settings changed meanwhile reached the test library only)
        prev.gsplat_set_quirks(quirks.get())
        prev.gsplat_set_deterministic(int(_DETERMINISTIC))


def hooks_active() -> bool:
    """True inside hooks(): the C ABI (and the torch op layer) run on the test library."""
    return _lib is not None and _lib is _hooks_lib


def variant_is_default() -> bool:
    """True while the shipped raster variants are selected (always in the shipped library)."""
    L = lib()
    return not hasattr(L, "gsplat_debug_raster_variant_is_default") or \
        bool(L.gsplat_debug_raster_variant_is_default())


def call(name: str, *args) -> int:
    """Call a status-returning entry point; non-zero status -> RuntimeError."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().gsplat_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed: {msg}")
    return rc


def call_status(name: str, *args) -> int:
    """Call an entry point whose non-zero statuses include expected outcomes (e.g.
    gsplat_bin_speculative's 2 = "needs I on the host"): the status is returned, not raised.
    (A separate function from call() so bench.py's per-entry timing sees it too.)"""
    return int(getattr(lib(), name)(*args))


def query(name: str, *args) -> int:
    """Call a size query (`*_workspace_size`)."""
    return int(getattr(lib(), name)(*args))


def ptr(t):
    """A tensor's device address for a `void *` argument (a plain int: ctypes converts it per
    the entry's argtypes, without a c_void_p object per argument)."""
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream(device) -> int:
    """The current HIP stream of `device`, as the `void *stream` argument (the raw handle
    straight from the stream registry: ~0.3 us instead of ~2.5 us for a torch.cuda.Stream
    object per call, tools/host_timeline.py)."""
    if _RAW_STREAM is not None:
        if not isinstance(device, (torch.device, int)):
            device = torch.device(device)
        idx = device.index if isinstance(device, torch.device) else device
        return _RAW_STREAM(torch.cuda.current_device() if idx is None else int(idx))
    return torch.cuda.current_stream(device).cuda_stream


def check_device(name: str, *tensors):
    """gsplat's CHECK_INPUT: ROCm-device, contiguous tensors only."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"{name}: expected a ROCm device tensor, got {t.device} "
                               "(this rasterizer has no CPU path)")
        if not t.is_contiguous():
            raise RuntimeError(f"{name}: tensor must be contiguous")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"{name}: tensors on different devices ({dev} vs {t.device})")
    return dev
