"""Loader of the schema-typed torch operator layer (csrc/torch_ops.cpp -> libgsplat_torch_ops.so).

`ops()` returns `torch.ops.gsplat_mi355x`, the TORCH_LIBRARY namespace whose ops wrap the
C-ABI launchers of libgsplat_mi355x.so (include/gsplat_mi355x.h) on the current HIP stream:

    project_fwd / project_bwd, sh_fwd / sh_bwd, map_intersects, sort_pairs, tile_bins,
    raster_fwd / raster_bwd

Each op has a Meta kernel, so graphs that call them trace under torch.compile / FakeTensor.
The C library is loaded through `_lib.lib()` first (quirks and determinism are set there);
the op library links the same file (rpath $ORIGIN), so both share one copy of its state.
There is no fallback: a missing library raises.
"""
from __future__ import annotations

import os

import torch

from . import _lib

OPS_PATH = os.environ.get("GSPLAT_MI355X_OPS_LIB") or os.path.join(_lib._HERE,
                                                                   "libgsplat_torch_ops.so")
OP_NAMES = ("project_fwd", "project_bwd", "sh_fwd", "sh_bwd", "map_intersects", "sort_pairs",
            "tile_bins", "raster_fwd", "raster_bwd")

_loaded = set()
# the op layer over the test library (_lib.hooks()): namespace gsplat_mi355x_hooks
OPS_HOOKS_PATH = os.path.join(_lib._HERE, "libgsplat_torch_ops_hooks.so")


def ops():
    """torch.ops.gsplat_mi355x, loading libgsplat_torch_ops.so on first use (inside
    _lib.hooks(): the copy over the test library, torch.ops.gsplat_mi355x_hooks)."""
    hooks = _lib.hooks_active()
    path = OPS_HOOKS_PATH if hooks else OPS_PATH
    if path not in _loaded:
        _lib.lib()
        if not os.path.exists(path):
            raise RuntimeError(
                f"gsplat MI355X torch op library not built: {path} is missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        torch.ops.load_library(path)
        _loaded.add(path)
    return torch.ops.gsplat_mi355x_hooks if hooks else torch.ops.gsplat_mi355x
