"""One switch for the gsplat 0.1.2.1 behaviours that SURVEY.md Appendix A recalls but could not
verify offline ([VERIFY]); include/gsplat_mi355x.h GSPLAT_QUIRK_* documents each bit.

  alpha_099      A10: the rasterize backward clamps alpha at 0.99 (the forward at 0.999)
  conic_half     A7/A9: v_conic.y = 1/2 v_sigma dx dy with the matching conic VJP (conics.grad
                 .y halves; means/scales/quats gradients are the same either way)
  ewa_unclamped  A6: the EWA VJP recomputes t without the 1.3 tan_fov clamp

GSPLAT_MI355X_QUIRKS selects them at import: "all" (default: gsplat as recalled), "none", or a
comma list of names (a leading "-" removes a name from all: "-ewa_unclamped").  Whoever holds
gsplat 0.1.2.1's source can pin parity by flipping the bits its kernels contradict.
"""
from __future__ import annotations

import os

ALPHA_099, CONIC_HALF, EWA_UNCLAMPED = 1, 2, 4
ALL = ALPHA_099 | CONIC_HALF | EWA_UNCLAMPED
NAMES = {"alpha_099": ALPHA_099, "conic_half": CONIC_HALF, "ewa_unclamped": EWA_UNCLAMPED}


def parse(spec) -> int:
    """A mask from an int, "all", "none" or a comma list of (optionally "-"-prefixed) names."""
    if isinstance(spec, int):
        if spec & ~ALL:
            raise ValueError(f"unknown quirk bits 0x{spec & ~ALL:x}")
        return spec
    spec = (spec or "all").strip().lower()
    if spec == "all":
        return ALL
    if spec == "none":
        return 0
    items = [s.strip() for s in spec.split(",") if s.strip()]
    mask = ALL if items and all(s.startswith("-") for s in items) else 0
    for s in items:
        name = s.lstrip("-")
        if name not in NAMES:
            raise ValueError(f"unknown quirk {name!r} (known: {', '.join(NAMES)})")
        mask = (mask & ~NAMES[name]) if s.startswith("-") else (mask | NAMES[name])
    return mask


_mask = parse(os.environ.get("GSPLAT_MI355X_QUIRKS", "all"))


def get() -> int:
    return _mask


def set(spec) -> int:
    """Select the quirks (mask, "all", "none" or names) for every later launch; returns the
    previous mask."""
    global _mask
    prev, _mask = _mask, parse(spec)
    from . import _lib
    if _lib._lib is not None:
        _lib.call("gsplat_set_quirks", _mask)
    return prev


def backward_alpha_clamp(mask=None) -> float:
    """alpha_max of the rasterize backward: 0.99 with A10, else the forward's 0.999."""
    return 0.99 if (get() if mask is None else mask) & ALPHA_099 else 0.999
