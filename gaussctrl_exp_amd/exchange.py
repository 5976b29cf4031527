"""Data-parallel gradient exchange for multi-view training.

Every rank renders its own camera(s) against the same replicated Gaussians, and the optimiser
needs the sum of the per-view gradients on every rank.  Of the 236 B of gradient per
Gaussian, 192 B are the SH coefficient gradient, and for one view that block is the
rank-1 product

    v_coeffs[i, k, c] = Y_k(means[i] - campos) * v_colors[i, c]

(gsplat 0.1.2.1 sh.cuh backward; viewdirs = means - camera centre, gc_model.py:197-200).
The means are replicated, so a view's whole SH gradient is determined by its v_colors
(12 B per Gaussian) and its camera centre.  `ShViewExchange` therefore all-gathers
[v_colors | campos] from every rank (one RCCL all-gather per view) and evaluates
sum_r Y(means - campos_r) (x) v_colors_r with one HIP kernel.  It sums in a fixed view
order, so every rank produces bit-identical coefficient gradients and the replicas stay in
sync.  At 8 ranks each GPU receives 7 x 12 B per Gaussian instead of ring-all-reducing 192 B
(2 x 7/8 x 192 B moved).  The other 44 B per Gaussian (means, scales, quats, opacities) are
all-reduced (the fused render issues that all-reduce from inside its backward).

Sparse records (the fused render): a view's colour gradient is exactly zero outside its
visible Gaussians (radii > 0), so when the views see a fraction of the scene (c4 garden: 55 %)
only the visible rows travel, after a visibility bitmap and its prefix (exchange_layout.h:
12 B per visible Gaussian + 0.19 B per Gaussian).  The ranks must agree on the record length:
the forward plans the bitmap as soon as radii exist and all-gathers the visible counts (async,
4 B per rank); the backward reads them (long arrived) and packs at capacity C = the largest
count, or packs the dense record when the sparse one would not be clearly smaller.  Sparse and
dense records give bit-identical sums (gsplat_compute_sh_backward_view_table).

Several views per rank per step (views_per_step > 1, TrainStep.forward_backward_views): each
view's record all-gather is issued from its own backward and left in flight while the rank
renders its next view; the geometry gradients accumulate in one flat buffer
(gsplat_fused_preprocess_backward_accumulate); the last view's backward issues the flat
all-reduce and evaluates every gathered record in one kernel.  Only the last view's exchange
is exposed, so the per-view exchange cost falls with the views per step.

Validity: the exchange assumes the SH coefficients reach the loss only through
`spherical_harmonics` -- true for the splatfacto / GaussCtrl caller (gc_model.py:190-204),
where features_dc / features_rest are concatenated and used nowhere else.  A caller that
adds another term on the coefficients (a regulariser, say) must use the plain all-reduce
(TrainStep(grad_exchange="allreduce")).
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import _lib

_ACTIVE: Optional["ShViewExchange"] = None

# a sparse record is used when it is at most this fraction of the dense one
SPARSE_MAX_FRAC = 0.9
# after a view whose agreed capacity leaves the sparse record above this fraction of the dense
# one, the next DENSE_SKIP views skip the plan and the count gather (dense records): the ranks
# share that history, so they skip together
DENSE_HOPELESS_FRAC = 0.95
DENSE_SKIP = 32
MAX_TABLE = 64  # exchange_layout.h XS_MAX_VIEWS: records per views kernel


def active() -> Optional["ShViewExchange"]:
    """The exchange a spherical_harmonics call made now should use in its backward."""
    return _ACTIVE


def sparse_floats(n: int, capacity: int) -> int:
    """Length in floats of a sparse view record of capacity `capacity` (exchange_layout.h)."""
    return 4 + 3 * ((n + 63) // 64) + 3 * capacity


class ShViewExchange:
    def __init__(self, group=None, sparse: str = "auto"):
        if sparse not in ("auto", "on", "off"):
            raise ValueError(f"sparse must be 'auto', 'on' or 'off', not {sparse}")
        self.group = group
        self.sparse = sparse
        self.means: Optional[torch.Tensor] = None
        self.campos: Optional[torch.Tensor] = None
        self.handled = False  # set when this step's SH gradient went through the exchange
        # the fused render's early all-reduce of the other four gradients (one flat buffer):
        # (async work, {param data_ptr: expected grad data_ptr})
        self.early = None
        self.early_steps = 0  # steps that took the early all-reduce (tests)
        self.views_per_step = 1
        self.view_index = 0
        self.pending = []  # this step's record gathers in flight: (work, out, floats, capacity)
        self.planned = {}  # view index -> (send buffer, count work, gathered counts)
        self.geo = None  # multi-view step: the flat geometry gradient summed over this rank's views
        self.record_kinds = {"sparse": 0, "dense": 0}  # views exchanged per record kind (tests)
        self.last_record_floats = None  # length of the last record sent (bench)
        self.last_capacity = None  # the agreed sparse capacity of the last planned view (bench)
        self._skip = 0  # views left to exchange dense without planning (DENSE_SKIP)
        # the SH-feature groups' Adam step fused into the views kernel (TrainStep sets it for
        # the step, reduce_views consumes it): dict(groups=[(param, exp_avg, exp_avg_sq, lr)] x 2
        # (features_dc, features_rest), step, betas, eps); adam_applied once the kernel ran
        self.adam = None
        self.adam_applied = False
        self._buffers = {}
        self._host_counts = None

    @contextlib.contextmanager
    def view(self, means: torch.Tensor, campos: torch.Tensor, index: int = 0, of: int = 1):
        # (set before the render, so a rank whose render never reaches spherical_harmonics
        #  can still take part in the step's exchange: TrainStep._null_sh_exchange)
        """Scope of one rank's render of view `index` of its `of` views this step: SH calls
        inside it exchange their gradients."""
        global _ACTIVE
        # every rank gathers world * of records into one table kernel: refuse a step that could
        # not be evaluated before any of its collectives is issued (not at the last view's
        # reduce_views, with the gathers and the geometry all-reduce already in flight)
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        if int(of) < 1 or world * int(of) > MAX_TABLE:
            raise ValueError(f"ShViewExchange: {world} ranks x {int(of)} views per step = "
                             f"{world * int(of)} records; the views kernel takes 1..{MAX_TABLE}")
        prev = _ACTIVE
        self.means = means.detach()
        self.campos = campos.detach().reshape(3).to(torch.float32)
        self.view_index, self.views_per_step = int(index), int(of)
        _ACTIVE = self
        try:
            yield self
        finally:
            _ACTIVE = prev

    @property
    def last_view(self) -> bool:
        return self.view_index + 1 >= self.views_per_step

    def reset(self):
        self.handled = False
        self.adam = None
        self.adam_applied = False
        self.early = None
        self.pending = []
        self.planned = {}
        self.geo = None

    def _buffer(self, key, numel, dev):
        b = self._buffers.get(key)
        if b is None or b.numel() < numel or b.device != dev:
            b = self._buffers[key] = torch.empty((numel,), device=dev, dtype=torch.float32)
        return b

    # ---- the caller path (spherical_harmonics backward) and the null record: dense, at once
    def gather(self, v_colors: torch.Tensor) -> torch.Tensor:
        """All ranks' [v_colors (3N floats) | campos (3) | pad] records, [world, 3N + 4]."""
        n = v_colors.shape[0]
        rec = torch.cat([v_colors.reshape(-1).float(), self.campos.to(v_colors.device),
                         torch.zeros(1, device=v_colors.device)])
        world = dist.get_world_size(self.group)
        out = torch.empty((world * (3 * n + 4),), device=v_colors.device, dtype=torch.float32)
        dist.all_gather_into_tensor(out, rec, group=self.group)
        return out.view(world, 3 * n + 4)

    def reduce(self, v_colors: Optional[torch.Tensor],
               views_backward: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]):
        """Summed coefficient gradient of all ranks' views (one view per rank, gathered now).
        `views_backward(means, views)` evaluates sum_r Y(means - campos_r) (x) v_colors_r from
        the gathered records."""
        views = self.gather(v_colors)
        self.handled = True
        return views_backward(self.means, views)

    # ---- the fused render: planned in the forward, packed after the raster backward --------
    def plan(self, n: int, radii: torch.Tensor, stream):
        """Forward, once radii exist: the visibility bitmap of this view's sparse record and the
        async all-gather of every rank's visible count."""
        dev = radii.device
        if self.sparse != "on" and (self.sparse == "off" or self._skip > 0):
            self._skip = max(self._skip - 1, 0)
            self.planned[self.view_index] = None  # dense record, no count gather
            return
        key = ("send", self.view_index)
        send = self._buffer(key, sparse_floats(n, n), dev)
        _lib.call("gsplat_exchange_sparse_plan", n, _lib.ptr(radii), _lib.ptr(send), stream)
        world = dist.get_world_size(self.group)
        counts = torch.empty((world,), device=dev, dtype=torch.float32)
        work = dist.all_gather_into_tensor(counts, send[3:4], group=self.group, async_op=True)
        self.planned[self.view_index] = (send, work, counts)

    def _capacity(self, dev) -> int:
        """The largest visible count over the ranks for the current view (host; the counts'
        all-gather was issued in the forward and has long completed)."""
        _, work, counts = self.planned[self.view_index]
        if self._host_counts is None or self._host_counts.numel() != counts.numel():
            self._host_counts = torch.empty((counts.numel(),), dtype=torch.int32,
                                            pin_memory=True)
        side = torch.cuda.Stream(dev) if not hasattr(self, "_side") else self._side
        self._side = side
        with torch.cuda.stream(side):
            work.wait()
            self._host_counts.copy_(counts.view(torch.int32), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        ev.synchronize()
        torch.cuda.current_stream(dev).wait_stream(side)
        return int(self._host_counts.max())

    def send_view(self, n: int, rec: torch.Tensor, radii: torch.Tensor, colors: torch.Tensor,
                  stream):
        """After the raster backward: pack this view's record (sparse at the agreed capacity, or
        dense) and issue its all-gather (async); reduce_views waits for it."""
        dev = rec.device
        campos = self.campos.to(dev).contiguous()
        planned = self.planned[self.view_index]
        dense_len = 3 * n + 4
        use_sparse = False
        if planned is not None:
            send = planned[0]
            cap = self._capacity(dev)
            self.last_capacity = cap
            use_sparse = self.sparse == "on" or (
                self.sparse == "auto" and sparse_floats(n, cap) <= SPARSE_MAX_FRAC * dense_len)
            if not use_sparse and sparse_floats(n, cap) > DENSE_HOPELESS_FRAC * dense_len:
                self._skip = DENSE_SKIP
        if use_sparse:
            length = sparse_floats(n, cap)
            _lib.call("gsplat_exchange_pack_sparse", n, _lib.ptr(rec), rec.numel(),
                      _lib.ptr(radii), _lib.ptr(colors), _lib.ptr(campos), _lib.ptr(send), cap,
                      stream)
            rec_send = send[:length]
        else:
            length, cap = dense_len, -1
            rec_send = self._buffer(("dense", self.view_index), dense_len, dev)[:dense_len]
            _lib.call("gsplat_exchange_pack_colors", n, _lib.ptr(rec), rec.numel(),
                      _lib.ptr(radii), _lib.ptr(colors), _lib.ptr(campos), _lib.ptr(rec_send),
                      stream)
        self.record_kinds["sparse" if use_sparse else "dense"] += 1
        self.last_record_floats = length
        world = dist.get_world_size(self.group)
        out = torch.empty((world * length,), device=dev, dtype=torch.float32)
        work = dist.all_gather_into_tensor(out, rec_send, group=self.group, async_op=True)
        self.pending.append((work, out, length, cap))
        del self.planned[self.view_index]

    def all_reduce_early(self, flat: torch.Tensor, early_map):
        """The fused render's flat geometry gradient (means/scales/quats/opacity, summed over
        this rank's views), all-reduced async; train.GradExchange then skips the four
        parameters (early_map: which gradient storage each parameter must hold) and waits."""
        self.early = (dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group,
                                      async_op=True), dict(early_map))
        self.early_steps += 1

    def reduce_views(self, degree: int, degrees_to_use: int):
        """(v_features_dc [N,3], v_features_rest [N,K-1,3]): the sum over every rank's views
        of this step, from the gathered records (view-major, rank order), in one kernel.  With
        `adam` set (TrainStep), that kernel applies the SH-feature groups' Adam step instead
        and (None, None) is returned."""
        means = self.means
        n = means.shape[0]
        dev = means.device
        ptrs, caps = [], []
        for work, out, length, cap in self.pending:
            work.wait()
            for r in range(out.numel() // length):
                ptrs.append(out.data_ptr() + 4 * r * length)
                caps.append(cap)
        if not ptrs or len(ptrs) > MAX_TABLE:
            raise RuntimeError(f"ShViewExchange: {len(ptrs)} gathered view records (1..{MAX_TABLE})")
        K = (degree + 1) ** 2
        R = len(ptrs)
        tab = (ctypes.c_void_p * R)(*ptrs)
        cap_arr = (ctypes.c_longlong * R)(*caps)
        means_c = means.float().contiguous()
        if self.adam is not None:
            # the SH-feature groups' Adam step inside the table kernel: parameters and moments
            # updated in place, no gradient tensors (gsplat_compute_sh_backward_view_table_adam)
            (pd, md, vd, lr_d), (pr, mr, vr, lr_r) = self.adam["groups"]
            b1, b2 = self.adam["betas"]
            P = _lib.ptr
            _lib.call("gsplat_compute_sh_backward_view_table_adam", n, degree,
                      int(degrees_to_use), R, P(means_c), ctypes.cast(tab, ctypes.c_void_p),
                      ctypes.cast(cap_arr, ctypes.c_void_p), P(pd), P(pr) if K > 1 else None,
                      P(md), P(vd), P(mr) if K > 1 else None, P(vr) if K > 1 else None,
                      float(lr_d), float(lr_r), int(self.adam["step"]), float(b1), float(b2),
                      float(self.adam["eps"]), _lib.stream(dev))
            self._last_gathered = [p[1] for p in self.pending]
            self.pending = []
            self.handled = True
            self.adam_applied = True
            return None, None
        v_dc = torch.empty((n, 3), device=dev, dtype=torch.float32)
        v_rest = torch.empty((n, K - 1, 3), device=dev, dtype=torch.float32)
        _lib.call("gsplat_compute_sh_backward_view_table", n, degree, int(degrees_to_use), R,
                  _lib.ptr(means_c), ctypes.cast(tab, ctypes.c_void_p),
                  ctypes.cast(cap_arr, ctypes.c_void_p), _lib.ptr(v_dc),
                  _lib.ptr(v_rest) if K > 1 else None, _lib.stream(dev))
        # (the gathered buffers must outlive the kernel: keep them until the next step)
        self._last_gathered = [p[1] for p in self.pending]
        self.pending = []
        self.handled = True
        return v_dc, v_rest
