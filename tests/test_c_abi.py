"""The C-ABI library loads and exports every entry point include/gsplat_mi355x.h declares
(no GPU needed: symbol resolution and pure host queries only), and the gsplat shim exposes
the gsplat 0.1.2.1 surface gc_model.py and splatfacto import."""
import ctypes
import inspect
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsplat_mi355x.h")


def _header_parts():
    """(shipped text, test-hook text) of the header: the declarations inside the
    `#ifdef GSPLAT_TEST_HOOKS` sections are the test library's only."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    hooks = "".join(re.findall(r"#ifdef GSPLAT_TEST_HOOKS(.*?)#endif", src, flags=re.S))
    shipped = re.sub(r"#ifdef GSPLAT_TEST_HOOKS.*?#endif", "", src, flags=re.S)
    return shipped, hooks


def _names(text):
    return sorted(set(re.findall(r"\b(gsplat_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    """The shipped library exports every declared entry point and none of the test hooks; the
    test library (GSPLAT_TEST_HOOKS) exports both; every declaration has a binding."""
    from gaussctrl_exp_amd import _lib
    shipped, hooks = _header_parts()
    names, hook_names = _names(shipped), _names(hooks)
    assert len(names) >= 18 and len(hook_names) >= 5
    lib = ctypes.CDLL(os.path.join(ROOT, "gaussctrl_exp_amd", "libgsplat_mi355x.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    leaked = [n for n in hook_names if hasattr(lib, n)]
    assert not leaked, leaked
    hl = ctypes.CDLL(_lib.HOOKS_PATH)
    missing = [n for n in names + hook_names if not hasattr(hl, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES)
    assert set(hook_names) == set(_lib.HOOK_SIGNATURES)


def _prototypes():
    """{name: parameter count} of every prototype in the header."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(gsplat_[a-z0-9_]+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_binding_arities_match_the_header():
    """ctypes argtypes have exactly as many entries as the C prototypes have parameters."""
    from gaussctrl_exp_amd import _lib
    protos = _prototypes()
    sigs = {**_lib.SIGNATURES, **_lib.HOOK_SIGNATURES}
    assert set(protos) == set(sigs)
    wrong = {n: (len(sigs[n][1]), k) for n, k in protos.items() if len(sigs[n][1]) != k}
    assert not wrong, wrong


def test_host_queries_without_gpu():
    from gaussctrl_exp_amd import _lib
    assert _lib.lib().gsplat_abi_version() == _lib.ABI_VERSION == 17
    assert _lib.query("gsplat_bin_count_workspace_size", 1000) > 1000 * 16
    assert _lib.query("gsplat_sort_isect_pairs_workspace_size", 0) > 0


def test_list_split_policy_without_gpu(hooks):
    """gsplat_rasterize_chunk_size: parts of ~0.6 mean list lengths (a multiple of 64, at least
    256) below 12,288 tiles, no split above (c5's 16,384 tiles) or without intersections; the
    debug override forces / disables it; the plan buffer grows with the part count."""
    from gaussctrl_exp_amd import _lib
    q = lambda *a: _lib.query("gsplat_rasterize_chunk_size", *a)
    assert q(68, 68, 7_717_748) == 1024  # headline: mean 1,669 per tile
    assert q(32, 32, 1_686_461) == 1024  # c3 bear: mean 1,647
    assert q(32, 32, 10_000) == 256      # short lists: the floor
    assert q(128, 128, 83_276_610) == 0  # c5: 16,384 tiles, unsplit
    assert q(32, 32, 0) == 0
    for t, i in ((68, 7_717_748), (32, 1_686_461), (50, 123_457)):
        c = q(t, t, i)
        assert c % 64 == 0 and c >= 256
    L = hooks
    try:
        L.gsplat_debug_set_chunk(100)
        assert q(68, 68, 7_717_748) == 128  # forced, rounded up to 64
        L.gsplat_debug_set_chunk(-1)
        assert q(68, 68, 7_717_748) == 0
    finally:
        L.gsplat_debug_set_chunk(0)
    b = lambda c: _lib.query("gsplat_rasterize_split_bytes", 68, 68, 7_717_748, c)
    assert b(0) == 0 and b(100) == 0  # no split / not a multiple of 64
    assert b(256) > b(1024) > 4624 * (4 + 8)  # work[T] + items[>= T]


def test_quirk_switch_reaches_the_library():
    """GSPLAT_MI355X_QUIRKS / quirks.set select the [VERIFY] behaviours in the library."""
    from gaussctrl_exp_amd import _lib, quirks
    L = _lib.lib()
    assert L.gsplat_get_quirks() == quirks.get()
    prev = quirks.set("none")
    try:
        assert L.gsplat_get_quirks() == 0 and quirks.backward_alpha_clamp() == 0.999
        quirks.set("-ewa_unclamped")
        assert L.gsplat_get_quirks() == quirks.ALPHA_099 | quirks.CONIC_HALF
        assert quirks.backward_alpha_clamp() == 0.99
        quirks.set("conic_half,ewa_unclamped")
        assert L.gsplat_get_quirks() == 6
        with pytest.raises(ValueError):
            quirks.set("no_such_quirk")
        with pytest.raises(RuntimeError, match="unknown bits"):
            _lib.call("gsplat_set_quirks", 8)
    finally:
        quirks.set(prev)
    assert L.gsplat_get_quirks() == prev


def test_bad_arguments_are_rejected_before_launch():
    from gaussctrl_exp_amd import _lib
    with pytest.raises(RuntimeError, match="bad sizes"):
        _lib.call("gsplat_rasterize_forward", 0, 1, 16, 16, 3, *([None] * 10), None)
    with pytest.raises(RuntimeError, match="bad args"):
        _lib.call("gsplat_compute_sh_forward", 10, 5, 1, None, None, None, None)


def test_gsplat_shim_surface():
    import gsplat
    from gsplat.project_gaussians import project_gaussians
    from gsplat.rasterize import rasterize_gaussians
    from gsplat.sh import num_sh_bases, spherical_harmonics
    assert [num_sh_bases(d) for d in range(5)] == [1, 4, 9, 16, 25]
    assert list(inspect.signature(project_gaussians).parameters) == [
        "means3d", "scales", "glob_scale", "quats", "viewmat", "projmat", "fx", "fy", "cx",
        "cy", "img_height", "img_width", "tile_bounds", "clip_thresh"]
    assert list(inspect.signature(rasterize_gaussians).parameters) == [
        "xys", "depths", "radii", "conics", "num_tiles_hit", "colors", "opacity",
        "img_height", "img_width", "background", "return_alpha"]
    assert list(inspect.signature(spherical_harmonics).parameters) == [
        "degrees_to_use", "viewdirs", "coeffs"]
    for name in ("map_gaussian_to_intersects", "bin_and_sort_gaussians",
                 "compute_cumulative_intersects", "compute_cov2d_bounds",
                 "get_tile_bin_edges", "ProjectGaussians", "RasterizeGaussians"):
        assert hasattr(gsplat, name)


def test_no_cpu_fallback():
    """The product path fails loudly on CPU tensors instead of silently computing."""
    from gaussctrl_exp_amd.camera import synthetic_camera
    from gaussctrl_exp_amd.project_gaussians import project_gaussians
    from gaussctrl_exp_amd.scene import synthetic_scene
    sc = synthetic_scene(10)
    cam = synthetic_camera(32, 32)
    with pytest.raises(RuntimeError, match="ROCm device"):
        project_gaussians(sc.means, torch.exp(sc.scales), 1, sc.quats, cam.viewmat,
                          cam.projmat, cam.fx, cam.fy, cam.cx, cam.cy, 32, 32,
                          cam.tile_bounds)


def test_rasterize_validates_shapes_like_gsplat():
    from gaussctrl_exp_amd.rasterize import rasterize_gaussians
    n = 4
    with pytest.raises(ValueError, match="xys must have dimensions"):
        rasterize_gaussians(torch.zeros(n, 3), torch.zeros(n), torch.zeros(n), torch.zeros(n, 3),
                            torch.zeros(n), torch.zeros(n, 3), torch.zeros(n, 1), 16, 16)
    with pytest.raises(ValueError, match="colors must have dimensions"):
        rasterize_gaussians(torch.zeros(n, 2), torch.zeros(n), torch.zeros(n), torch.zeros(n, 3),
                            torch.zeros(n), torch.zeros(n), torch.zeros(n, 1), 16, 16)


def test_emit_capacity_clamped_to_the_c_limit():
    """the pre-launch capacity is I + I/8 but never above the capacity
    gsplat_bin_emit_prelaunch accepts (bin_emit_impl rejects > 0x3FFFFFFF), so a frame shape
    whose I lies just under the limit keeps working on later calls."""
    from gaussctrl_exp_amd import _lib
    from gaussctrl_exp_amd.rasterize import EMIT_CAP_MAX, emit_capacity
    assert EMIT_CAP_MAX == 0x3FFFFFFF
    assert emit_capacity(0) == 0
    assert emit_capacity(8_000_000) == 9_000_000
    for I in (955_000_000, 1_000_000_000, 0x3FFFFFFF):
        assert emit_capacity(I) == EMIT_CAP_MAX
    # the C ABI sizes a workspace for that capacity (a pure host query, no GPU)
    assert _lib.query("gsplat_bin_emit_workspace_size_for", 1000, EMIT_CAP_MAX, 68, 68) > 0
