"""Differentiable tile rasterizer (gsplat 0.1.2.1 `gsplat/rasterize.py`).

`rasterize_gaussians` is called by /root/reference/gaussctrl/gc_model.py:208-220 (RGB with
return_alpha=True, random background during training) and :225-236 (depth, eval).  The
binning (cumsum -> intersect map -> sort -> tile bins) runs fused on the GPU
(csrc/binning.hip) with one host read of the intersection count, exactly where gsplat
reads `cum_tiles_hit[-1].item()`; blending runs in csrc/raster.hip.

The eval render calls rasterize_gaussians twice on the same projected Gaussians (RGB, then
depth as colours).  The binning depends only on (xys, depths, radii, num_tiles_hit, H, W),
so the second call reuses the first call's binning (`_BinCache`) when those are the very
same live tensors, unmodified, on the same stream.  `rasterize_gaussians_rgbd` goes further:
RGB, depth and alpha from one binning and one traversal.
"""
from __future__ import annotations

import collections
import os
import time
import weakref
from typing import Optional

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib, quirks
from .ops import ops

BLOCK_X, BLOCK_Y = 16, 16


def rasterize_gaussians(
    xys: Tensor,
    depths: Tensor,
    radii: Tensor,
    conics: Tensor,
    num_tiles_hit: Tensor,
    colors: Tensor,
    opacity: Tensor,
    img_height: int,
    img_width: int,
    background: Optional[Tensor] = None,
    return_alpha: Optional[bool] = False,
):
    """Rasterize 2D Gaussians by front-to-back alpha blending per 16x16 tile.

    Args: xys [N,2], depths [N], radii [N] int, conics [N,3], num_tiles_hit [N] int (all
    from project_gaussians), colors [N,C] (float, or uint8 -> /255), opacity [N,1],
    img_height, img_width, background [C] (default ones), return_alpha.

    Returns out_img [H,W,C], plus out_alpha [H,W] = 1 - final transmittance when
    return_alpha.  Gradients flow to xys, conics, colors and opacity.
    """
    if colors.dtype == torch.uint8:
        # make sure colors are float [0,1]
        colors = colors.float() / 255

    if background is not None:
        assert background.shape[0] == colors.shape[-1], (
            f"incorrect shape of background color tensor, expected shape {colors.shape[-1]}")
    else:
        background = torch.ones(colors.shape[-1], dtype=torch.float32, device=colors.device)

    if xys.ndimension() != 2 or xys.size(1) != 2:
        raise ValueError("xys must have dimensions (N, 2)")

    if colors.ndimension() != 2:
        raise ValueError("colors must have dimensions (N, D)")

    return _RasterizeGaussians.apply(
        xys.contiguous(), depths.contiguous(), radii.contiguous(), conics.contiguous(),
        num_tiles_hit.contiguous(), colors.contiguous(), opacity.contiguous(), img_height,
        img_width, background.contiguous(), return_alpha)


class _CountSlots:
    """Pinned host words the binning kernels write the (visible count, intersection count) of
    one call into (pinned host memory is device-addressable on ROCm).  Every bin_gaussians
    call takes a slot of its own for as long as it waits, so calls in flight on different
    streams or threads never share a word: a queued scan of one call cannot overwrite the
    count another call is polling."""

    SLOTS = 64

    def __init__(self):
        import threading
        self.lock = threading.Lock()
        self.bufs = {}
        self.busy = {}
        self.last_visible = {}

    def acquire(self, dev):
        with self.lock:
            if dev not in self.bufs:
                buf = torch.zeros((self.SLOTS, 4), dtype=torch.int32, pin_memory=True)
                self.bufs[dev] = (buf, buf.numpy())
                self.busy[dev] = set()
            busy = self.busy[dev]
            free = next((k for k in range(self.SLOTS) if k not in busy), None)
            if free is None:
                raise RuntimeError(f"bin_gaussians: more than {self.SLOTS} calls in flight")
            busy.add(free)
            buf, host = self.bufs[dev]
            host[free, :2] = -1
            host[free, 2:] = 0  # (gsplat_bin_count_keyed_ex: violation flag, varying key bits)
            return free, buf[free], host[free]

    def release(self, dev, slot, visible=None):
        with self.lock:
            self.busy[dev].discard(slot)
            if visible is not None:
                self.last_visible[dev] = visible


_COUNTS = _CountSlots()


def last_num_visible(dev) -> int:
    """The visible-Gaussian count of this device's last completed bin_gaussians call (written
    by the binning next to the intersection count)."""
    return int(_COUNTS.last_visible.get(dev, 0))


def _wait_count(host, dev, spin_s: float = 2.0) -> int:
    """The single host sync of the binning (gsplat: cum_tiles_hit[-1].item()): the scan kernel
    writes the intersection count once, straight into this call's pinned slot, so the host
    polls that word (about a microsecond from the write to the read) instead of a copy kernel
    plus a stream synchronisation (tens of microseconds of wake-up latency).  Falls back to
    synchronising the stream the binning was issued on (dev's current stream) if nothing
    arrives within spin_s."""
    t_end = None
    while True:
        v = int(host[1])
        if v != -1:
            return v
        if t_end is None:
            t_end = time.perf_counter() + spin_s
        elif time.perf_counter() > t_end:
            torch.cuda.current_stream(dev).synchronize()
            v = int(host[1])
            if v == -1:
                raise RuntimeError("bin_gaussians: the intersection count was never written")
            return v


def bin_gaussians(xys: Tensor, depths: Tensor, radii: Tensor, num_tiles_hit: Tensor,
                  img_height: int, img_width: int, keyed_workspace: Optional[Tensor] = None):
    """Fused on-device binning: (num_intersects, gaussian_ids_sorted [I] int32,
    tile_bins [tiles, 2] int32).  Same order as gsplat's stable-sorted isect_ids.
    keyed_workspace: a gsplat_bin_count workspace gsplat_fused_preprocess_forward_binned
    already filled with the depth-sort inputs (the depth-key pass is skipped)."""
    n = xys.shape[0]
    tbx = (img_width + BLOCK_X - 1) // BLOCK_X
    tby = (img_height + BLOCK_Y - 1) // BLOCK_Y
    dev = xys.device
    radii = radii.to(torch.int32).contiguous()
    num_tiles_hit = num_tiles_hit.to(torch.int32).contiguous()
    depths = depths.float().contiguous()
    xys = xys.float().contiguous()
    _lib.check_device("bin_gaussians", xys, depths, radii, num_tiles_hit)
    if n == 0:
        return 0, torch.empty((0,), device=dev, dtype=torch.int32), \
            torch.zeros((tbx * tby, 2), device=dev, dtype=torch.int32)
    P, st = _lib.ptr, _lib.stream(dev)
    tile_bins = torch.empty((tbx * tby, 2), device=dev, dtype=torch.int32)
    slot, counts, host = _COUNTS.acquire(dev)
    visible = None
    try:
        if keyed_workspace is not None:
            ws1 = keyed_workspace
            # (no pass skipped: learns the depth keys' varying bits for the speculative calls)
            _lib.call("gsplat_bin_count_keyed_ex", n, tbx, tby, P(counts), P(ws1), ws1.numel(),
                      0, st)
        else:
            ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=dev,
                              dtype=torch.uint8)
            _lib.call("gsplat_bin_count", n, P(xys), P(depths), P(radii), P(num_tiles_hit), tbx,
                      tby, P(counts), P(ws1), ws1.numel(), st)
        # the phase-2 outputs are allocated while the count phase runs, sized by the last
        # intersection count of this frame shape (+1/8), and the part of the emission that needs
        # only phase 1 is launched into them before the host waits for I: the GPU works through
        # the host's read of I and its launch of the rest instead of idling
        key = (dev, n, tbx, tby)
        cap = _EMIT_CAP.get(key, 0)
        pre = None
        if cap:
            pre = _emit_buffers(dev, n, cap, tbx, tby)
        if cap and PRELAUNCH_EMISSION:
            _lib.call("gsplat_bin_emit_prelaunch", n, cap, tbx, tby, P(tile_bins), P(ws1),
                      ws1.numel(), P(pre[1]), pre[1].numel(), st)
        num_intersects = _wait_count(host, dev)
        visible = int(host[0])
        if keyed_workspace is not None:
            _note_key_range(key, host)
    finally:
        _COUNTS.release(dev, slot, visible)
    _note_capacity(key, num_intersects)
    if pre is not None and num_intersects <= cap and not PRELAUNCH_EMISSION:  # (A/B runs)
        ids_buf, ws2 = pre
        _lib.call("gsplat_bin_emit", n, num_intersects, tbx, tby, P(ids_buf), P(tile_bins),
                  P(ws1), ws1.numel(), P(ws2), ws2.numel(), st)
    elif pre is not None and num_intersects <= cap:
        ids_buf, ws2 = pre
        _lib.call("gsplat_bin_emit_finish", n, num_intersects, cap, tbx, tby, P(ids_buf),
                  P(tile_bins), P(ws1), ws1.numel(), P(ws2), ws2.numel(), st)
    else:  # first call of this frame shape, or more intersections than the capacity
        ids_buf, ws2 = _emit_buffers(dev, n, num_intersects, tbx, tby)
        _lib.call("gsplat_bin_emit", n, num_intersects, tbx, tby, P(ids_buf), P(tile_bins),
                  P(ws1), ws1.numel(), P(ws2), ws2.numel(), st)
    return num_intersects, ids_buf[:max(num_intersects, 0)], tile_bins


class SpeculativeBinning:
    """A binning whose emission and tile sort were launched at a capacity before the host knew
    the intersection count I (gsplat_bin_emit_speculative): the caller launches the blend right
    behind it and calls finish() only then, so the GPU never idles at the host's read of I.

    ids (capacity slots; [0, I) valid) and tile_bins are the binning's outputs once finish()
    returns True; False means I exceeded the capacity -- the table was left all-zero (the blend
    behind it rendered the background) and the caller re-bins with rebin() and re-launches.
    `layout_intersects` is the count the list-split plan layout must use (both the forward that
    fills a plan and its backward): the capacity, known before I."""

    def __init__(self, dev, n, tbx, tby, ws1, slot, counts, host, key, cap, ids, ws2,
                 tile_bins):
        self.dev, self.n, self.tbx, self.tby = dev, n, tbx, tby
        self.ws1, self.slot, self.counts, self.host, self.key = ws1, slot, counts, host, key
        self.cap, self.ids, self.ws2, self.tile_bins = cap, ids, ws2, tile_bins
        self.layout_intersects = cap
        self.num_intersects = None
        self.range_violated = False

    def finish(self) -> bool:
        visible = None
        try:
            I = _wait_count(self.host, self.dev)
            visible = int(self.host[0])
            # a depth-sort digit assumed constant from earlier calls varied: the order is wrong
            # (the caller re-runs the preprocess -- the sort consumed its keys -- and re-bins)
            self.range_violated = int(self.host[2]) != 0
            _note_key_range(self.key, self.host)
        finally:
            _COUNTS.release(self.dev, self.slot, visible)
        self.num_intersects = I
        if not self.range_violated:  # (a violated sort's I is meaningless: the caller re-bins)
            _note_capacity(self.key, I)
        return I <= self.cap and not self.range_violated

    def rebin(self):
        """After an overflow (not a range violation): the emission and tile sort for the exact I
        (phase 1's workspace is untouched by the speculative launch) -> (ids [I], tile_bins)."""
        assert not self.range_violated
        I = self.num_intersects
        P, st = _lib.ptr, _lib.stream(self.dev)
        ids_buf, ws2 = _emit_buffers(self.dev, self.n, I, self.tbx, self.tby)
        _lib.call("gsplat_bin_emit", self.n, I, self.tbx, self.tby, P(ids_buf),
                  P(self.tile_bins), P(self.ws1), self.ws1.numel(), P(ws2), ws2.numel(), st)
        self.ids, self.ws2, self.cap = ids_buf, ws2, I
        self.layout_intersects = I
        return ids_buf[:I], self.tile_bins


def speculative_capacity(n: int, img_height: int, img_width: int, dev) -> int:
    """The capacity (intersection layout) bin_gaussians_speculative will use for this frame
    shape, or 0 when it will not run speculatively (first call of the shape, switched off)."""
    if n == 0 or not SPECULATIVE_BINNING:
        return 0
    tbx = (img_width + BLOCK_X - 1) // BLOCK_X
    tby = (img_height + BLOCK_Y - 1) // BLOCK_Y
    return _EMIT_CAP.get((dev, n, tbx, tby), 0)


def bin_gaussians_speculative(xys: Tensor, depths: Tensor, radii: Tensor, num_tiles_hit: Tensor,
                              img_height: int, img_width: int,
                              keyed_workspace: Optional[Tensor] = None, between=None):
    """bin_gaussians without the host read of I in the middle: the count phase, then -- when
    this frame shape's capacity is known from an earlier call and the binning scheme allows it
    -- the emission and the whole tile sort at that capacity (gsplat_bin_emit_speculative).
    Returns a SpeculativeBinning (finish() before using I), or None when the capacity is not
    known yet or the scheme needs I on the host (the caller then uses bin_gaussians).
    between: called between the count phase (the depth sort) and the emission + tile sort,
    which then go out as two C-ABI calls (the sorted scheme, uses_tile_sort); with the tile
    buckets, or on the fallback paths, it is called once after the binning's launches instead
    -- always before this function returns, so work it issues precedes any blend."""
    n = xys.shape[0]
    tbx = (img_width + BLOCK_X - 1) // BLOCK_X
    tby = (img_height + BLOCK_Y - 1) // BLOCK_Y
    dev = xys.device
    key = (dev, n, tbx, tby)
    cap = _EMIT_CAP.get(key, 0)
    if n == 0 or cap <= 0 or keyed_workspace is None or not SPECULATIVE_BINNING:
        return None
    _lib.check_device("bin_gaussians_speculative", xys, depths, radii, num_tiles_hit)
    P, st = _lib.ptr, _lib.stream(dev)
    ws1 = keyed_workspace
    tile_bins = torch.empty((tbx * tby, 2), device=dev, dtype=torch.int32)
    ids_buf, ws2 = _emit_buffers(dev, n, cap, tbx, tby)
    slot, counts, host = _COUNTS.acquire(dev)
    try:
        # the count phase and the tile sort in one call
        assume = _assumed_constant(key)
        if between is not None and uses_tile_sort(n, tbx * tby):
            _lib.call("gsplat_bin_count_keyed_ex", n, tbx, tby, P(counts), P(ws1), ws1.numel(),
                      assume, st)
            between()
            between = None
            rc = _lib.call_status("gsplat_bin_emit_speculative", n, cap, tbx, tby, P(ids_buf),
                                  P(tile_bins), P(ws1), ws1.numel(), P(ws2), ws2.numel(), st)
            if rc != 0:
                raise RuntimeError("gsplat_bin_emit_speculative failed (" + str(rc) + "): " +
                                   _lib.lib().gsplat_last_error().decode(errors="replace"))
        else:
            rc = _lib.call_status("gsplat_bin_speculative", n, cap, tbx, tby, P(counts), P(ws1),
                                  ws1.numel(), assume, P(ids_buf), P(tile_bins),
                                  P(ws2), ws2.numel(), st)
        if rc == 2:  # the scheme needs I on the host: count, then finish as bin_gaussians does
            _lib.call("gsplat_bin_count_keyed_ex", n, tbx, tby, P(counts), P(ws1), ws1.numel(),
                      _assumed_constant(key), st)
            pre = (ids_buf, ws2)
            if PRELAUNCH_EMISSION:
                _lib.call("gsplat_bin_emit_prelaunch", n, cap, tbx, tby, P(tile_bins), P(ws1),
                          ws1.numel(), P(ws2), ws2.numel(), st)
            I = _wait_count(host, dev)
            violated = int(host[2]) != 0
            _note_key_range(key, host)
            _COUNTS.release(dev, slot, int(host[0]))
            slot = None
            if violated:  # (an assumed-constant depth digit varied: the caller starts over)
                # the caller may blend before it calls finish(): nothing was emitted, so the
                # table must read as empty (it was uninitialised here)
                tile_bins.zero_()
                done = SpeculativeBinning(dev, n, tbx, tby, ws1, None, None, None, key, cap,
                                          ids_buf, ws2, tile_bins)
                done.num_intersects, done.range_violated = I, True
                done.finish = lambda: False
                if between is not None:
                    between()
                return done
            _note_capacity(key, I)
            if I <= cap:
                _lib.call("gsplat_bin_emit_finish", n, I, cap, tbx, tby, P(pre[0]), P(tile_bins),
                          P(ws1), ws1.numel(), P(pre[1]), pre[1].numel(), st)
                ids_buf, ws2 = pre
            else:
                ids_buf, ws2 = _emit_buffers(dev, n, I, tbx, tby)
                _lib.call("gsplat_bin_emit", n, I, tbx, tby, P(ids_buf), P(tile_bins), P(ws1),
                          ws1.numel(), P(ws2), ws2.numel(), st)
            done = SpeculativeBinning(dev, n, tbx, tby, ws1, None, None, None, key,
                                      max(I, cap), ids_buf, ws2, tile_bins)
            done.num_intersects = I
            done.layout_intersects = I
            done.finish = lambda: True
            if between is not None:
                between()
            return done
        if rc != 0:
            raise RuntimeError("gsplat_bin_speculative failed: " +
                               _lib.lib().gsplat_last_error().decode(errors="replace"))
    except BaseException:
        if slot is not None:
            _COUNTS.release(dev, slot)
        raise
    sb = SpeculativeBinning(dev, n, tbx, tby, ws1, slot, counts, host, key, cap, ids_buf, ws2,
                            tile_bins)
    if between is not None:  # (one call: the work goes after the binning's launches)
        between()
    return sb


# the tile buckets' size limit (binning.hip use_bucket: N <= 2^17 takes them, on at most
# BK_MAX_BUCKETS - 1 tiles)
BUCKET_MAX_N = 1 << 17
BK_MAX_BUCKETS = 16448


def uses_tile_sort(n: int, tiles: int) -> bool:
    """binning.hip use_bucket's complement for the shipped dispatch: the depth sort + tile sort
    (two-call speculative binning possible) rather than the tile buckets."""
    return n > BUCKET_MAX_N or tiles + 1 > BK_MAX_BUCKETS
# frame shape -> the intersection capacity to pre-allocate the emission's outputs for
_EMIT_CAP = {}
# frame shape -> the intersection counts of its last CAP_WINDOW binnings: the capacity is 1/8
# above their maximum, so a training loop that draws a random camera each step
# (gc_datamanager.py:218) overflows only on a view with more intersections than any of the last
# CAP_WINDOW (round 4 sized it from the previous frame alone: every larger view re-binned)
_CAP_WINDOW = {}
CAP_WINDOW = 64
# speculative binnings of the fused render: calls, and those that had to re-bin (capacity
# overflow / a depth digit assumed constant that varied) -- bench.py's speculative_misses
SPEC_STATS = {"speculative": 0, "overflow": 0, "range": 0, "sync": 0}


def _note_capacity(key, num_intersects: int):
    w = _CAP_WINDOW.get(key)
    if w is None:
        w = _CAP_WINDOW[key] = collections.deque(maxlen=CAP_WINDOW)
    w.append(int(num_intersects))
    _EMIT_CAP[key] = emit_capacity(max(w))
# frame shape -> the depth-key bits seen varying over the visible Gaussians (the union over
# calls, from gsplat_bin_count_keyed_ex's d_counts[3]); the speculative binning skips the
# depth-sort passes whose digit lies in the complement (GSPLAT_MI355X_ASSUME_RANGE=0: never)
_KEY_VARY = {}
ASSUME_KEY_RANGE = os.environ.get("GSPLAT_MI355X_ASSUME_RANGE", "1") != "0"


def _note_key_range(key, host):
    _KEY_VARY[key] = _KEY_VARY.get(key, 0) | (int(host[3]) & 0xFFFFFFFF)


def _assumed_constant(key) -> int:
    v = _KEY_VARY.get(key)
    return 0 if v is None or not ASSUME_KEY_RANGE else (~v) & 0xFFFFFFFF
# the fused render bins speculatively (bin_gaussians_speculative); GSPLAT_MI355X_SPECULATIVE=0
# turns it off (A/B runs)
SPECULATIVE_BINNING = os.environ.get("GSPLAT_MI355X_SPECULATIVE", "1") != "0"
# the C ABI's bound on an emission capacity (bin_emit_impl rejects larger ones)
EMIT_CAP_MAX = 0x3FFFFFFF


def emit_capacity(num_intersects: int) -> int:
    """The next call's pre-launch capacity after a call with `num_intersects`: 1/8 headroom,
    clamped to what gsplat_bin_emit_prelaunch accepts (an unclamped I + I/8 above
    the C limit made every later call of that frame shape fail)."""
    return max(0, min(num_intersects + (num_intersects >> 3), EMIT_CAP_MAX))
# launch the emission's first part before the host reads I (False: after it; A/B runs only)
PRELAUNCH_EMISSION = True


def _emit_buffers(dev, n, cap, tbx, tby):
    ids = torch.empty((max(cap, 0),), device=dev, dtype=torch.int32)
    ws2 = torch.empty((_lib.query("gsplat_bin_emit_workspace_size_for", n, cap, tbx, tby),),
                      device=dev, dtype=torch.uint8)
    return ids, ws2


class _BinCache:
    """The last rasterize call's binning, reused while its inputs are the same tensor
    objects (weak references: a freed tensor whose address is recycled never matches),
    at the same version counter (an in-place edit invalidates), size and stream."""

    def __init__(self):
        self.refs = None
        self.key = None
        self.value = None
        self.hits = 0

    @staticmethod
    def _key(tensors, H, W, stream):
        return (tuple((t._version, tuple(t.shape), t.dtype) for t in tensors), H, W,
                stream)

    def get(self, tensors, H, W, stream):
        if self.refs is None or len(self.refs) != len(tensors):
            return None
        if any(r() is not t for r, t in zip(self.refs, tensors)):
            return None
        if self.key != self._key(tensors, H, W, stream):
            return None
        self.hits += 1
        return self.value

    def put(self, tensors, H, W, stream, value):
        self.refs = [weakref.ref(t) for t in tensors]
        self.key = self._key(tensors, H, W, stream)
        self.value = value

    def clear(self):
        self.refs = self.key = self.value = None


_BIN_CACHE = _BinCache()


class _KeyedWorkspaces:
    """The depth-sort inputs project_gaussians wrote for its latest outputs
    (gsplat_project_gaussians_forward_binned), handed to the rasterize call that bins exactly
    those outputs -- the same tensor objects (weak references), unmodified (version counters),
    for the same tile grid, on the same stream.  Single use: the sort consumes the workspace.

    The entry never outlives its key: it is dropped when taken, when the binning cache
    answers the rasterize call instead (_binning), and when the projection outputs it was
    written for are freed (a finalizer on xys) -- so an unrasterized projection does not pin
    the ~60 B/Gaussian workspace."""

    def __init__(self):
        self.cache = _BinCache()
        self.serial = 0

    def put(self, tensors, tbx, tby, ws1):
        self.cache.put(tensors, tbx, tby, _lib.stream(tensors[0].device), ws1)
        self.serial += 1
        weakref.finalize(tensors[0], self._expire, self.serial)

    def _expire(self, serial):
        if serial == self.serial:
            self.cache.clear()

    def take(self, tensors, tbx, tby, stream):
        ws1 = self.cache.get(tensors, tbx, tby, stream)
        if ws1 is not None:
            self.cache.clear()
        return ws1


keyed_workspaces = _KeyedWorkspaces()


def _binning(xys, depths, radii, num_tiles_hit, H, W):
    """bin_gaussians through the one-entry cache (see module docstring), with the depth-sort
    inputs the projection kernel already wrote when these are its outputs."""
    key_tensors = (xys, depths, radii, num_tiles_hit)
    st = _lib.stream(xys.device)
    hit = _BIN_CACHE.get(key_tensors, H, W, st)
    tbx, tby = (W + BLOCK_X - 1) // BLOCK_X, (H + BLOCK_Y - 1) // BLOCK_Y
    if hit is not None:
        keyed_workspaces.take(key_tensors, tbx, tby, st)  # (unused: release it)
        return hit
    ws1 = keyed_workspaces.take(key_tensors, tbx, tby, st)
    res = bin_gaussians(xys, depths, radii, num_tiles_hit, H, W, keyed_workspace=ws1)
    _BIN_CACHE.put(key_tensors, H, W, st, res)
    return res


def rasterize_gaussians_rgbd(xys: Tensor, depths: Tensor, radii: Tensor, conics: Tensor,
                             num_tiles_hit: Tensor, colors: Tensor, opacity: Tensor,
                             img_height: int, img_width: int,
                             background: Optional[Tensor] = None):
    """Fused eval render: (rgb [H,W,3], depth [H,W,1], alpha [H,W]) from one
    binning and one traversal.  rgb and alpha equal rasterize_gaussians(..., return_alpha=True);
    depth equals channel 0 of rasterize_gaussians(..., colors=depths[:, None].repeat(1, 3),
    background=zeros(3)) -- gc_model.py:225-236's second call -- before the caller's division
    by alpha.  Forward only (no autograd): the eval path runs without gradients."""
    H, W = int(img_height), int(img_width)
    if colors.dim() != 2 or colors.shape[-1] != 3:
        raise ValueError("rasterize_gaussians_rgbd: colors must be [N, 3]")
    num_points = xys.size(0)
    tbx = (W + BLOCK_X - 1) // BLOCK_X
    tby = (H + BLOCK_Y - 1) // BLOCK_Y
    with torch.no_grad():
        xys, conics = xys.float().contiguous(), conics.float().contiguous()
        colors, opacity = colors.float().contiguous(), opacity.float().contiguous()
        depths_f = depths.float().contiguous()
        if background is None:
            background = torch.ones(3, dtype=torch.float32, device=colors.device)
        background = background.float().contiguous()
        dev = _lib.check_device("rasterize_gaussians_rgbd", xys, depths_f, radii, conics,
                                num_tiles_hit, colors, opacity, background)
        if opacity.numel() != num_points or conics.shape != (num_points, 3) or \
                colors.shape[0] != num_points or depths_f.numel() != num_points:
            raise ValueError("rasterize_gaussians_rgbd: inconsistent per-Gaussian tensor shapes")
        num_intersects, gaussian_ids_sorted, tile_bins = _binning(xys, depths, radii,
                                                                  num_tiles_hit, H, W)
        if num_intersects < 1:
            return (torch.ones(H, W, 3, device=dev) * background,
                    torch.zeros(H, W, 1, device=dev), torch.ones(H, W, device=dev))
        out_img = torch.empty((H, W, 3), device=dev, dtype=torch.float32)
        out_depth = torch.empty((H, W, 1), device=dev, dtype=torch.float32)
        final_Ts = torch.empty((H, W), device=dev, dtype=torch.float32)
        final_idx = torch.empty((H, W), device=dev, dtype=torch.int32)
        P = _lib.ptr
        _lib.call("gsplat_rasterize_forward_rgbd", tbx, tby, H, W, P(gaussian_ids_sorted),
                  P(tile_bins), P(xys), P(conics), P(colors), P(depths_f), P(opacity),
                  P(background), P(out_img), P(out_depth), P(final_Ts), P(final_idx),
                  _lib.stream(dev))
        return out_img, out_depth, 1 - final_Ts


class _RasterizeGaussians(Function):
    """Rasterizes 2D gaussians (autograd wrapper of the C-ABI binning/raster kernels)."""

    @staticmethod
    def forward(ctx, xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height,
                img_width, background=None, return_alpha=False):
        num_points = xys.size(0)
        H, W = int(img_height), int(img_width)
        tbx = (W + BLOCK_X - 1) // BLOCK_X
        tby = (H + BLOCK_Y - 1) // BLOCK_Y
        C = colors.shape[-1]
        xys, conics = xys.float().contiguous(), conics.float().contiguous()
        colors, opacity = colors.float().contiguous(), opacity.float().contiguous()
        background = background.float().contiguous()
        dev = _lib.check_device("rasterize_gaussians", xys, depths, radii, conics,
                                num_tiles_hit, colors, opacity, background)
        if opacity.numel() != num_points or conics.shape != (num_points, 3) or \
                colors.shape[0] != num_points:
            raise ValueError("rasterize_gaussians: inconsistent per-Gaussian tensor shapes")

        num_intersects, gaussian_ids_sorted, tile_bins = _binning(
            xys, depths, radii, num_tiles_hit, H, W)

        if num_intersects < 1:
            # gsplat 0.1.x: background image, final_Ts zero (so alpha = 1)
            out_img = torch.ones(H, W, C, device=dev) * background
            final_Ts = torch.zeros(H, W, device=dev)
            final_idx = torch.zeros(H, W, device=dev, dtype=torch.int32)
        else:
            P = _lib.ptr
            if C == 3 and any(ctx.needs_input_grad) and \
                    _lib.variant_is_default():
                # the backward accumulates into per-Gaussian gradient records that this blend
                # zeroes as its waves finish (no memset in the backward; every record, since
                # gsplat_grad_records_split reads the culled Gaussians' zeros too)
                out_img = torch.empty((H, W, C), device=dev, dtype=torch.float32)
                final_Ts = torch.empty((H, W), device=dev, dtype=torch.float32)
                final_idx = torch.empty((H, W), device=dev, dtype=torch.int32)
                rec = torch.empty((_lib.query("gsplat_grad_records_bytes", num_points),),
                                  device=dev, dtype=torch.uint8)
                _lib.call("gsplat_rasterize_forward_clearing", tbx, tby, H, W,
                          P(gaussian_ids_sorted), P(tile_bins), P(xys), P(conics), P(colors),
                          P(opacity), P(background), P(out_img), P(final_Ts), P(final_idx),
                          P(rec), rec.numel(), None, 0, 0, None, 0, _lib.stream(dev))
                ctx.rec = rec
            else:
                out_img, final_Ts, final_idx = ops().raster_fwd(
                    tbx, tby, H, W, gaussian_ids_sorted, tile_bins, xys, conics, colors,
                    opacity, background)
        if not hasattr(ctx, "rec"):
            ctx.rec = None

        ctx.img_width = W
        ctx.img_height = H
        ctx.num_intersects = num_intersects
        ctx.opacity_shape = opacity.shape
        ctx.save_for_backward(gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                              background, final_Ts, final_idx)
        ctx.set_materialize_grads(False)  # an unused alpha output costs no zero fill

        if return_alpha:
            out_alpha = 1 - final_Ts
            return out_img, out_alpha
        return out_img

    @staticmethod
    def backward(ctx, v_out_img, v_out_alpha=None):
        H, W = ctx.img_height, ctx.img_width
        (gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background, final_Ts,
         final_idx) = ctx.saved_tensors
        num_points, C = colors.shape
        dev = xys.device
        if v_out_img is None:
            v_out_img = torch.zeros((H, W, C), device=dev, dtype=torch.float32)

        if ctx.num_intersects < 1:
            v_xy = torch.zeros_like(xys)
            v_conic = torch.zeros_like(conics)
            v_colors = torch.zeros_like(colors)
            v_opacity = torch.zeros_like(opacity)
        else:
            v_out_img = v_out_img.float().contiguous()
            if v_out_alpha is not None:  # NULL = zero alpha gradient
                v_out_alpha = v_out_alpha.float().contiguous()
            tbx = (W + BLOCK_X - 1) // BLOCK_X
            tby = (H + BLOCK_Y - 1) // BLOCK_Y
            # list-split backward (C = 3): the plan buffer its first two kernels fill
            chunk = _lib.query("gsplat_rasterize_chunk_size", tbx, tby, ctx.num_intersects) \
                if C == 3 else 0
            if ctx.rec is None and chunk == 0:  # plain list walk: the torch op layer
                v_xy, v_conic, v_colors, v_opacity = ops().raster_bwd(
                    tbx, tby, H, W, gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                    background, final_Ts, final_idx, v_out_img, v_out_alpha,
                    quirks.backward_alpha_clamp())
                return (v_xy, None, None, v_conic, None, v_colors,
                        v_opacity.view(ctx.opacity_shape), None, None, None, None)
            v_xy = torch.empty((num_points, 2), device=dev, dtype=torch.float32)
            v_conic = torch.empty((num_points, 3), device=dev, dtype=torch.float32)
            v_colors = torch.empty((num_points, C), device=dev, dtype=torch.float32)
            v_opacity = torch.empty(ctx.opacity_shape, device=dev, dtype=torch.float32)
            P = _lib.ptr
            plan = torch.empty((max(_lib.query("gsplat_rasterize_split_bytes", tbx, tby,
                                               ctx.num_intersects, chunk), 1),),
                               device=dev, dtype=torch.uint8)
            plan_bytes = plan.numel() if chunk > 0 else 0
            st = _lib.stream(dev)
            if ctx.rec is not None:  # records cleared by the forward blend
                rec = ctx.rec
                _lib.call("gsplat_rasterize_backward_records", tbx, tby, H, W, num_points,
                          P(gaussian_ids_sorted), P(tile_bins), P(xys), P(conics), P(colors),
                          P(opacity), P(background), P(final_Ts), P(final_idx), P(v_out_img),
                          P(v_out_alpha), quirks.backward_alpha_clamp(), ctx.num_intersects,
                          chunk, P(plan), plan_bytes, 0, P(rec), rec.numel(), st)
                _lib.call("gsplat_grad_records_split", num_points, P(rec), rec.numel(),
                          P(conics), P(opacity), P(v_xy), P(v_conic), P(v_colors), P(v_opacity),
                          st)
                ctx.rec = None
                return (v_xy, None, None, v_conic, None, v_colors, v_opacity, None, None, None,
                        None)
            wsz = _lib.query("gsplat_rasterize_backward_workspace_size", num_points, C)
            ws = torch.empty((max(wsz, 1),), device=dev, dtype=torch.uint8)
            _lib.call("gsplat_rasterize_backward_chunked", tbx, tby, H, W, num_points,
                      P(gaussian_ids_sorted), P(tile_bins), P(xys), P(conics), P(colors),
                      P(opacity), P(background), P(final_Ts), P(final_idx), P(v_out_img),
                      P(v_out_alpha), quirks.backward_alpha_clamp(), P(v_xy), P(v_conic),
                      P(v_colors), P(v_opacity), ctx.num_intersects, chunk, P(plan),
                      plan_bytes, P(ws), wsz, st)

        return (
            v_xy,  # xys
            None,  # depths
            None,  # radii
            v_conic,  # conics
            None,  # num_tiles_hit
            v_colors,  # colors
            v_opacity,  # opacity
            None,  # img_height
            None,  # img_width
            None,  # background
            None,  # return_alpha
        )
