#!/usr/bin/env python3
"""Headline benchmark: differentiable 3DGS rasterizer fwd+bwd on MI355X.

BASELINE.json metric: "Mpixels/s fwd+bwd and train iters/s, 1M Gaussians @ 1080^2".

A step = one view per GPU: project -> SH (deg 3) -> bin/sort -> rasterize forward ->
loss -> backward through rasterize / SH / project, plus (N > 1) the RCCL all-reduce of the
Gaussian gradients -- the multi-view exchange of the data-parallel train step
(SURVEY.md §8e).  `value` = all ranks' rendered pixels / max-over-ranks step time.  The
full train step (splatfacto 0.8 L1 + 0.2 SSIM loss + Adam) is timed separately and
reported as `train_iters_per_s`.  Inputs are synthetic (SURVEY.md §8d scene: random
Gaussians in [-1.5,1.5]^3 seen from (0,0,4), fov 50 deg) and resident in HBM before timing.
`roofline` describes the dominant entry (HBM fraction plus its PMC issue / wait shares);
`lane_occupancy` gives the blend kernels' live and valid-pair shares of their lane slots,
counted on one extra, untimed step.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config headline|c2|c3|c4|c5]
(N > 1 under torch.distributed.run, one process per GPU, backend nccl = RCCL.)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gaussctrl_exp_amd import _lib, timing  # noqa: E402
from gaussctrl_exp_amd.camera import gc_camera, look_at_c2w  # noqa: E402
from gaussctrl_exp_amd.fused import render_fused  # noqa: E402
from gaussctrl_exp_amd import rasterize  # noqa: E402
from gaussctrl_exp_amd.rasterize import bin_gaussians  # noqa: E402
from gaussctrl_exp_amd.scene import render, synthetic_scene  # noqa: E402
from gaussctrl_exp_amd.sh import num_sh_bases  # noqa: E402
from gaussctrl_exp_amd.train import TrainStep  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# untimed steps before the first timed leg (clock settle, see main); reported as settle_steps
SETTLE_STEPS = 40

CONFIGS = {
    # name: (N, W, H, sh_degree, scale_lo, scale_hi, seed, real scene or None, description)
    "headline": (1_000_000, 1080, 1080, 3, 0.005, 0.02, 10, None,
                 "1M synthetic Gaussians @ 1080x1080, SH deg 3, fwd+bwd"),
    "c2": (100_000, 512, 512, 0, 0.005, 0.03, 2, None,
           "100k synthetic Gaussians @ 512x512, SH deg 0, forward rasterize only"),
    "c3": (300_000, 512, 512, 3, 0.0025, 0.012, 3, "bear",
           "bear: 300k Gaussians seeded around data/bear/sparse_pc.ply (34,174 points), "
           "bear cameras (transforms.json, 512x512), SH deg 3, fwd+bwd"),
    "c4": (2_000_000, 1080, 1080, 3, 0.0016, 0.006, 4, "garden",
           "garden: 2M Gaussians seeded around data/garden/sparse_pc.ply (27,046 points), "
           "garden cameras rescaled x1080/512, 1 view/GPU (first sorted frames), SH deg 3, "
           "fwd+bwd"),
    "c5": (5_000_000, 2048, 2048, 3, 0.01, 0.016, 5, None,
           "5M synthetic Gaussians @ 2048x2048, SH deg 3, heavy overlap, fwd+bwd"),
}


FORWARD_ONLY = {"c2"}  # BASELINE.json configs[1]: "forward rasterize only"


def make_workload(config: str, rank: int, dev):
    """(scene, camera) of one rank.  Synthetic configs: SURVEY.md §8d scene, camera `rank`
    of an orbit.  Real configs: Gaussians seeded around the scene's sparse point cloud and
    the scene's own camera `rank` (dataparser coordinates; tests/golden fixtures written by
    tools/make_scene_fixtures.py, so the GPU box needs no reference checkout)."""
    N, W, H, deg, lo, hi, seed, real, _ = CONFIGS[config]
    if real is None:
        return synthetic_scene(N, deg, seed=seed, scale_lo=lo, scale_hi=hi, device=dev), \
            view_camera(W, H, rank)
    import numpy as np
    from gaussctrl_exp_amd.formats import load_transforms, transform_points
    from gaussctrl_exp_amd.scene import scene_from_points
    golden = os.path.join(ROOT, "tests", "golden")
    d = load_transforms(os.path.join(golden, f"{real}_transforms.json"))
    pc = np.load(os.path.join(golden, f"{real}_sparse_pc.npz"))
    pts = transform_points(torch.from_numpy(pc["xyz"]), d.transform_matrix, d.points_scale)
    scene = scene_from_points(pts, torch.from_numpy(pc["rgb"]), N, deg, seed=seed,
                              scale_lo=lo, scale_hi=hi, device=dev)
    return scene, config_camera(config, rank)


def config_camera(config: str, index: int):
    """Camera `index` of `config`: the synthetic orbit's view, or the real scene's own camera
    (dataparser coordinates, rescaled to the config's width)."""
    N, W, H, deg, lo, hi, seed, real, _ = CONFIGS[config]
    if real is None:
        return view_camera(W, H, index)
    from gaussctrl_exp_amd.formats import load_transforms, rescale_cameras
    d = load_transforms(os.path.join(ROOT, "tests", "golden", f"{real}_transforms.json"))
    cam = d.cameras[index % len(d.cameras)]
    if cam.width != W:
        cam = rescale_cameras([cam], W / cam.width)[0]
    return cam


def view_camera(W, H, view: int):
    """Camera `view` of an orbit at radius 4 around the origin (view 0 = (0,0,4))."""
    ang = 2 * math.pi * view / 8.0
    eye = (4.0 * math.sin(ang), 0.3 * math.sin(3 * ang), 4.0 * math.cos(ang))
    fx = 0.5 * W / math.tan(math.radians(25.0))
    return gc_camera(look_at_c2w(eye, up=(0.0, 1.0, 0.0)), fx, fx, W / 2.0, H / 2.0, W, H)


def algorithmic_bytes(N, I, P, T, K, nvis):
    """Per-view algorithmic HBM bytes of each C-ABI entry point (SURVEY.md §8d model; the
    binning entries count every radix pass's key/value reads and writes)."""
    tile_passes = max(1, -(-max(1, (T - 1).bit_length()) // 8))  # 8-bit digits of the tile id
    # the tile buckets (shipped for N <= 2^17 on <= 16,447 tiles; the test library's
    # gsplat_debug_binning_scheme can force either scheme)
    L = _lib.lib()
    setting = int(L.gsplat_debug_binning_scheme(-2)) if \
        hasattr(L, "gsplat_debug_binning_scheme") else -1
    bucket = setting == 1 or (setting == -1 and N <= (1 << 17) and T + 1 <= 16448)
    if bucket:
        # count: allotment + visibility sums over the records and keys (20 N); emit: the
        # records twice (bucket counts, placement: 32 N), ids placed (4 I), then per tile the ids
        # and their depth keys read and the sorted ids written (12 I), the tile table (8 T)
        bin_count, bin_emit = 20 * N, 32 * N + 16 * I + 8 * T
        emit_head = 32 * N + 4 * I  # pre-launched: counts, scan, placement
    else:
        # depth keys (44 N) + 4 radix passes (count 4 N, scatter 16 N each) + the depth-ordered
        # record gather (36 N) + the allotment scan (8 N); keyed: without the key pass
        # emission (records in, (tile, id) pairs out) + per tile-digit pass 20 I + bin edges
        bin_count, bin_emit = 168 * N, 20 * N + 8 * I + 20 * tile_passes * I + 4 * I + 8 * T
        # pre-launched: the emission (none when the first tile pass is generated, I >= 2^24)
        emit_head = 0 if I >= (1 << 24) else 20 * N + 8 * I
    return {
        "gsplat_project_gaussians_forward": 96 * N,
        "gsplat_compute_sh_forward": (24 + 12 * K) * N,
        "gsplat_bin_count": bin_count,
        "gsplat_bin_count_keyed": bin_count if bucket else bin_count - 44 * N,
        "gsplat_bin_count_keyed_ex": bin_count if bucket else bin_count - 44 * N,
        # count + emission + tile sort in one call (the speculative binning)
        "gsplat_bin_speculative": (bin_count if bucket else bin_count - 44 * N) + bin_emit,
        "gsplat_bin_emit": bin_emit,
        # the emission split around the host's read of I (rasterize.bin_gaussians)
        "gsplat_bin_emit_prelaunch": emit_head,
        "gsplat_bin_emit_finish": bin_emit - emit_head,
        "gsplat_rasterize_forward": 40 * I + 20 * P,
        "gsplat_rasterize_backward": 40 * I + 24 * P + 36 * N,
        "gsplat_compute_sh_backward": (24 + 12 * K) * N,
        "gsplat_project_gaussians_backward": 180 * N,
        # fused training render (csrc/preprocess.hip): raw params (56 + 12 (K-1) B) in,
        # projection + colour + opacity (48 B) out
        "gsplat_fused_preprocess_forward": (92 + 12 * K) * N,
        # + the binning's depth key, id and 16-B record per Gaussian
        "gsplat_fused_preprocess_forward_binned": (116 + 12 * K) * N,
        # its two parts (round 4: the colours on a second stream): params + projection outputs
        # + binning inputs; means, features and colours
        "gsplat_fused_preprocess_forward_part[1]": 104 * N,
        "gsplat_fused_preprocess_forward_part[2] (side stream)": (24 + 12 * K) * N,
        # its blend also zeroes the 48-B gradient record of every visible Gaussian
        "gsplat_rasterize_forward_clearing": 40 * I + 20 * P + 48 * nvis,
        "gsplat_rasterize_backward_records": 40 * I + 24 * P,
        # the fused L1 loss (round 4): the forward also reads gt (12 P); the backward reads the
        # image and gt (24 P) in place of v_out / v_alpha (16 P), + final T and index (8 P)
        "gsplat_rasterize_forward_clearing_l1": 40 * I + 32 * P + 48 * nvis,
        "gsplat_rasterize_backward_records_l1": 40 * I + 32 * P,
        # params + saved forward outputs (72 B) and the 48 B record in, 6 gradients out
        "gsplat_fused_preprocess_backward": (116 + 12 * K) * N + 48 * nvis,
        # the same with the Adam step inside (one GPU): no gradients written; every parameter
        # and its two moments read and written (24 B per parameter, 11 + 3 K per Gaussian)
        "gsplat_fused_preprocess_backward_adam": (72 + 24 * (11 + 3 * K)) * N + 48 * nvis,
        # the splatfacto loss (loss.hip): forward reads pred + gt and writes the three SSIM
        # derivative maps (60 P); backward reads the maps, pred and gt, writes v_pred (72 P)
        "gsplat_l1_ssim_forward": 60 * P,
        "gsplat_l1_ssim_backward": 72 * P,
        # standalone multi-tensor Adam (N > 1): param, grad, m, v in; param, m, v out
        "gsplat_adam_step": 28 * (11 + 3 * K) * N,
    }


# train_roofline: which part of the train step each C-ABI entry belongs to (SURVEY.md §8d asks
# for the step's byte split: render vs loss vs Adam vs the exchange)
def train_part(entry: str) -> str:
    if entry.startswith("gsplat_l1_ssim"):
        return "loss"
    if entry == "gsplat_adam_step":
        return "adam"
    if entry == "gsplat_fused_preprocess_backward_adam":
        return "geometry backward + adam (one kernel)"
    if entry == "gsplat_compute_sh_backward_view_table_adam":
        return "exchange: multi-view SH backward + SH-feature Adam (one kernel)"
    if entry.startswith("gsplat_exchange") or "views" in entry or "view_table" in entry:
        return "exchange (pack / multi-view SH backward)"
    return "render"


# Device kernels behind each C-ABI entry (for the PMC counters of the dominant entry), and
# whether their loads are 16-B-per-lane streaming reads -- the only access width for which
# MI355X_MICROARCH.md calibrates gfx950's FETCH_SIZE (it reports half the bytes: x2).  The
# blend kernels gather 4-8 B per lane; their FETCH_SIZE is reported raw (uncalibrated).
ENTRY_KERNELS = {
    "gsplat_rasterize_backward": (("raster_bwd", "split_grads_kernel"), False),
    "gsplat_rasterize_backward_records": (("raster_bwd",), False),
    "gsplat_rasterize_backward_records_l1": (("raster_bwd",), False),
    "gsplat_rasterize_forward_clearing_l1": (("raster_fwd", "post_forward"), False),
    "gsplat_fused_preprocess_forward": (("fused_fwd_kernel",), True),
    "gsplat_fused_preprocess_forward_binned": (("fused_fwd_kernel",), True),
    "gsplat_fused_preprocess_forward_part[1]": (("fused_fwd_proj_kernel",), True),
    "gsplat_fused_preprocess_forward_part[2] (side stream)": (("fused_fwd_sh_kernel",), True),
    # (a pattern's '&'-separated parts must all occur in the instantiation's name)
    "gsplat_fused_preprocess_backward": (("fused_bwd_kernel&, false>",), True),
    "gsplat_fused_preprocess_backward_adam": (("fused_bwd_kernel&, true>",), True),
    "gsplat_l1_ssim_forward": (("l1_ssim_fwd_kernel", "l1_ssim_finalize"), False),
    "gsplat_l1_ssim_backward": (("l1_ssim_bwd_kernel",), False),
    "gsplat_rasterize_forward": (("raster_fwd",), False),
    "gsplat_rasterize_forward_clearing": (("raster_fwd",), False),
    "gsplat_compute_sh_forward": (("sh_fwd_kernel",), True),
}
PMC_TRAFFIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                           "pmc_traffic.json")


def _pmc_entry(entry, config):
    """Per-call counter sums of a C-ABI entry whose kernels the PMC summary attributed by
    dispatch order (the binning: tools/pmc_summary.py), or None."""
    try:
        with open(PMC_TRAFFIC) as f:
            return json.load(f)["configs"][config]["entries"][entry]
    except (OSError, ValueError, KeyError):
        return None


def _pmc_kernels(config):
    """The committed rocprofv3 PMC summary of `config` (profiles/pmc_traffic.json, written by
    tools/pmc_bench.sh + tools/pmc_summary.py on that config), or None: counters collected on
    another config are never used."""
    try:
        with open(PMC_TRAFFIC) as f:
            return json.load(f)["configs"][config]["kernels"]
    except (OSError, ValueError, KeyError):
        return None


def _entry_kernel_rows(entry, config):
    """The PMC rows of an entry's kernels on `config`: per kernel pattern of ENTRY_KERNELS, the
    most-dispatched instantiation matching it (the one the timed step launches; the bench's
    other legs -- deterministic, unchanged-caller, warm-up variants -- run other instantiations
    far fewer times), keyed by the full instantiation name (tools/kname.py).  [] without that
    config's counters."""
    kern = _pmc_kernels(config)
    pats, _ = ENTRY_KERNELS.get(entry, ((), False))
    if not kern or not pats:
        return []
    out = []
    for p in pats:
        parts = p.split("&")
        cand = [(v.get("dispatches") or 0.0, name) for name, v in kern.items()
                if all(q in name for q in parts)]
        if cand:
            name = max(cand)[1]
            if all(name != n for n, _ in out):
                out.append((name, kern[name]))
    return out


def pmc_traffic(entry, config):
    """HBM bytes per call of a C-ABI entry on `config`: FETCH_SIZE (x2 only for streaming
    16-B-per-lane kernels, see ENTRY_KERNELS) + WRITE_SIZE; None without counters."""
    e = _pmc_entry(entry, config)
    if e and e.get("fetch_kb") is not None:  # binning entries: raw FETCH_SIZE (gathers)
        return int((e["fetch_kb"] + (e.get("write_kb") or 0.0)) * 1024.0)
    _, streaming = ENTRY_KERNELS.get(entry, ((), False))
    tot, hit = 0.0, False
    for name, v in _entry_kernel_rows(entry, config):
        if v.get("fetch_kb") is not None:
            tot += ((2.0 if streaming else 1.0) * v["fetch_kb"] + (v.get("write_kb") or 0.0)) \
                * 1024.0
            hit = True
    return int(tot) if hit else None


def pmc_valu_busy(entry, config, ms_per_call, n_simd=256 * 4, clock_hz=2.4e9):
    """rocprofv3 SQ_ACTIVE_INST_VALU (counted in quad-cycles) per call / (SIMDs x call duration
    in quad-cycles at the peak engine clock): the VALU pipe's active share if every wave64 VALU
    op held it for 4 cycles.  gfx950's 32-lane SIMD issues one in 2 (MI355X_MICROARCH.md), so
    this overstates the issue share ~2x; valu_issue_frac (pmc_issue_and_wait) is the issue
    bound, wait_frac the stall share.  None without that config's counters."""
    e = _pmc_entry(entry, config)
    if e and e.get("valu_quad_cycles") is not None and ms_per_call:
        return round(e["valu_quad_cycles"] / (n_simd * ms_per_call * 1e-3 * clock_hz / 4.0), 3)
    if not ms_per_call:
        return None
    tot, hit = 0.0, False
    for name, v in _entry_kernel_rows(entry, config):
        if v.get("valu_quad_cycles") is not None:
            tot += v["valu_quad_cycles"]
            hit = True
    return round(tot / (n_simd * ms_per_call * 1e-3 * clock_hz / 4.0), 3) if hit else None


def pmc_issue_and_wait(entry, config, ms_per_call, n_simd=256 * 4, clock_hz=2.4e9):
    """(valu_issue_frac, wait_frac, issue_stall_frac) of the entry's kernels on `config`: the
    lower bound on the SIMD issue cycles its VALU instructions take -- SQ_INSTS_VALU x 2 cycles
    (a wave64 VALU op issues over 2 cycles on gfx950's 32-lane SIMD) + SQ_INSTS_VALU_TRANS_F32
    x 2 more (a transcendental takes 4), packed ops counted at the scalar cost -- per
    SIMD-cycle of the call; SQ_WAIT_ANY / SQ_WAVE_CYCLES, the share of its waves' lifetime
    parked on s_waitcnt / barriers; SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, the share spent ready but
    not issuing (dependency / pipe / arbitration stalls; MI355X_MICROARCH.md counter table).
    Nones without that config's counters."""
    e = _pmc_entry(entry, config)
    if e and e.get("insts_valu") is not None:
        rows = [e]
    else:
        rows = [v for _, v in _entry_kernel_rows(entry, config) if v.get("insts_valu") is not None]
    if not rows or not ms_per_call:
        return None, None, None
    iv = sum(v["insts_valu"] for v in rows)
    it = sum(v.get("insts_trans") or 0.0 for v in rows)
    wa = sum(v.get("wait_any") or 0.0 for v in rows)
    wi = sum(v.get("wait_inst_any") or 0.0 for v in rows)
    wc = sum(v.get("wave_cycles") or 0.0 for v in rows)
    issue = (2.0 * iv + 2.0 * it) / (n_simd * ms_per_call * 1e-3 * clock_hz)
    has_wa = any(v.get("wait_any") is not None for v in rows)
    return (round(issue, 3), (round(wa / wc, 3) if wc and has_wa else None),
            (round(wi / wc, 3) if wc else None))


def pmc_insts_valu(entry, config):
    """SQ_INSTS_VALU (wave64 VALU instructions) per call of the entry's kernels on `config` -- the
    instantiations the timed step ran (_entry_kernel_rows) -- or None without that config's
    counters."""
    vals = [v["insts_valu"] for _, v in _entry_kernel_rows(entry, config)
            if v.get("insts_valu") is not None]
    return sum(vals) if vals else None


def lane_occupancy(step, dev, config):
    """Lane-slot accounting of the blend kernels over one extra step (outside every timed
    region), from the counting instantiations behind gsplat_debug_pair_count: per kernel the
    share of the pixel slots its wave iterations issue whose pixel is still live for the staged
    Gaussian (inside the image, not terminated / idx <= final_idx) and the share holding a
    valid pixel-Gaussian pair (sigma >= 0, alpha >= 1/255 as well) -- the work the VALU-bound
    blend loops actually do -- plus, where that config's PMC is committed, wave64 VALU
    instructions x 64 per valid pair."""
    buf = torch.zeros(6, dtype=torch.int64, device=dev)
    _lib.call("gsplat_debug_pair_count", _lib.ptr(buf))
    try:
        step()
        torch.cuda.synchronize()
    finally:
        _lib.call("gsplat_debug_pair_count", None)
    c = buf.tolist()
    out = {}
    for entry, (s, live, valid) in (("gsplat_rasterize_backward_records", c[0:3]),
                                    ("gsplat_rasterize_forward_clearing", c[3:6])):
        if not s:
            continue
        iv = pmc_insts_valu(entry, config)
        out[entry] = {
            "lane_slots": s,
            "live_frac": round(live / s, 4),
            "valid_pair_frac": round(valid / s, 4),
            "valu_lane_ops_per_valid_pair": round(iv * 64 / valid, 1) if iv and valid else None,
        }
    return out


def cpu_threads():
    """Host threads the CPU baseline may use: the CPUs this process may run on, capped by
    OMP_NUM_THREADS when the job sets it (the GPU box gives one GPU's job 16 of its CPUs
    and says so there; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(scene, cam, sh_degree, n_tiles=256, seed=0, backward=True):
    """The north-star CPU baseline: a naive pure-PyTorch per-pixel rasterizer
    (oracle/torch_ref.render_fwd_bwd_sampled: gc_model's activations, projection, SH,
    torch.sort binning, per-pixel compositing over each tile's whole list, autograd backward)
    on all host threads, the compositing timed on `n_tiles` seeded random tiles and
    extrapolated by the tile count.  The single-threaded C oracle (a hand-written port of
    gsplat's kernels, a much stronger CPU program) is timed on 64 tiles beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_ref as TR
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        sc = scene.detach().to("cpu")
        H, W = cam.height, cam.width
        T = cam.tile_bounds[0] * cam.tile_bounds[1]
        total, d = TR.render_fwd_bwd_sampled(
            sc.means, sc.scales, sc.quats, sc.opacities, sc.features_dc, sc.features_rest,
            cam.viewmat, cam.projmat, cam.c2w[:3, 3], cam.fx, cam.fy, cam.cx, cam.cy, H, W,
            sh_degree, n_tiles=min(n_tiles, T), seed=seed, backward=backward)
    finally:
        torch.set_num_threads(prev)
    c_port = c_oracle_baseline(scene, cam, sh_degree, seed=seed) if backward else None
    return {
        "value": round(H * W / total / 1e6, 5),
        "unit": "Mpixels/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"pure-PyTorch per-pixel rasterizer (oracle/torch_ref.py), "
                   f"{'fwd + autograd bwd' if backward else 'forward only'}, torch.set_num_threads({threads}) (host os.cpu_count()="
                   f"{os.cpu_count()}): per-Gaussian stages over all {sc.means.shape[0]} "
                   f"Gaussians + torch.sort binning of {d['intersects']} intersections "
                   f"({d['t_gauss']:.2f}s) + compositing fwd+bwd on {d['tiles']} of {T} random "
                   f"tiles ({d['t_tiles']:.2f}s) extrapolated x{d['scale']:.1f}; "
                   f"est {total:.1f}s per view"),
        "c_oracle_1thread": c_port,
    }


def c_oracle_baseline(scene, cam, sh_degree, budget_tiles=64, seed=0):
    """C oracle (single-threaded restatement of gsplat) on a bounded sample: the full
    per-Gaussian stages (project, SH, map+stable sort+bins) plus rasterize fwd+bwd on
    `budget_tiles` random tiles, extrapolated to all tiles."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    rng = np.random.default_rng(seed)
    sc = scene.detach().to("cpu")
    means = sc.means.numpy()
    scales = torch.exp(sc.scales).numpy()
    quats = (sc.quats / sc.quats.norm(dim=-1, keepdim=True)).numpy()
    opac = torch.sigmoid(sc.opacities).numpy()
    coeffs = torch.cat([sc.features_dc[:, None], sc.features_rest], 1).numpy()
    H, W = cam.height, cam.width
    t0 = time.perf_counter()
    xys, depths, radii, conics, nth, cov3d = O.project_forward(
        means, scales, 1.0, quats, cam.viewmat.numpy(), cam.projmat.numpy(), cam.fx, cam.fy,
        cam.cx, cam.cy, H, W, cam.tile_bounds)
    dirs = means - cam.c2w[:3, 3].numpy()
    dirs = dirs / np.linalg.norm(dirs, axis=1, keepdims=True)
    colors = np.maximum(O.sh_forward(sh_degree, dirs, coeffs) + 0.5, 0.0).astype(np.float32)
    b = O.bin_and_sort(xys, depths, radii, nth, cam.tile_bounds)
    t_gauss_fwd = time.perf_counter() - t0
    T = cam.tile_bounds[0] * cam.tile_bounds[1]
    tiles = rng.choice(T, size=min(budget_tiles, T), replace=False).astype(np.int32)
    bg = np.zeros(3, np.float32)
    t0 = time.perf_counter()
    img, fT, fi = O.rasterize_forward(cam.tile_bounds, H, W, b["gaussian_ids_sorted"],
                                      b["tile_bins"], xys, conics, colors, opac, bg,
                                      tile_list=tiles)
    v_img = np.ones((H, W, 3), np.float32)
    v_a = np.zeros((H, W), np.float32)
    gr = O.rasterize_backward(cam.tile_bounds, H, W, b["gaussian_ids_sorted"], b["tile_bins"],
                              xys, conics, colors, opac, bg, fT, fi, v_img, v_a,
                              tile_list=tiles)
    t_tiles = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.sh_backward(sh_degree, dirs, gr[2], coeffs.shape[1])
    O.project_backward(means, scales, 1.0, quats, cam.viewmat.numpy(), cam.projmat.numpy(),
                       cam.fx, cam.fy, cam.cx, cam.cy, H, W, cov3d, radii, conics, gr[0],
                       np.zeros_like(depths), gr[1])
    t_gauss_bwd = time.perf_counter() - t0
    total = t_gauss_fwd + t_gauss_bwd + t_tiles * T / len(tiles)
    return {
        "value": round(H * W / total / 1e6, 4),
        "unit": "Mpixels/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"C oracle, 1 thread: full project+SH+bin/sort+SH-bwd+project-bwd over "
                   f"{means.shape[0]} Gaussians ({t_gauss_fwd + t_gauss_bwd:.2f}s) + rasterize "
                   f"fwd+bwd on {len(tiles)} of {T} random tiles ({t_tiles:.2f}s) "
                   f"extrapolated x{T / len(tiles):.1f}; est {total:.1f}s per view"),
    }


def view_cameras(config: str, rank: int, dev, count: int = 16):
    """The cameras a training loop would draw for `config`, in the order it would draw them:
    synthetic configs cycle the 8-view orbit from view `rank`; real configs draw the scene's own
    training cameras at random (gc_datamanager.py:218: a random camera each step; seeded per
    rank), rescaled to the config's width."""
    N, W, H, deg, lo, hi, seed, real, _ = CONFIGS[config]
    if real is None:
        return [view_camera(W, H, (rank + k) % 8).to(dev) for k in range(count)]
    import random
    from gaussctrl_exp_amd.formats import load_transforms, rescale_cameras
    d = load_transforms(os.path.join(ROOT, "tests", "golden", f"{real}_transforms.json"))
    rng = random.Random(1234 + rank)
    cams = []
    for _ in range(count):
        c = d.cameras[rng.randrange(len(d.cameras))]
        if c.width != W:
            c = rescale_cameras([c], W / c.width)[0]
        cams.append(c.to(dev))
    return cams


def rotating_cameras(config, rank, dev, step, timed, steps, world):
    """The timed step under the reference's camera pattern: the same step with
    a different camera each step (view_cameras), after one warm-up pass over them.  A camera
    change can defeat what the speculative binning learns from earlier frames (the capacity:
    a running maximum over the shape's recent intersection counts; the depth-key bits seen
    varying): speculative_misses counts the steps that had to re-bin."""
    cams = view_cameras(config, rank, dev)
    state = {"i": 0}

    def rot():
        step(c=cams[state["i"] % len(cams)])
        state["i"] += 1
    for _ in range(len(cams)):
        rot()
    torch.cuda.synchronize()
    s0 = dict(rasterize.SPEC_STATS)
    dt = timed(rot, steps)
    H, W = cams[0].height, cams[0].width
    s1 = rasterize.SPEC_STATS
    return {"value": round(world * H * W * steps / dt / 1e6, 2),
            "misses": {k: s1[k] - s0[k] for k in s1},
            "desc": (f"{len(cams)} cameras cycled: " +
                     ("the 8-view orbit" if CONFIGS[config][7] is None else
                      f"random draws from the {CONFIGS[config][7]} training cameras"))}


def exchange_profile(scene, cam, gt, bg, deg, world, dev, steps, timed, record_floats=None):
    """N > 1 only: what the data-parallel exchange costs this rank and how much of it the step
    hides.  Times (max over ranks, same `steps`): the step's compute alone (the
    same render + loss + backward on a world-size-1 TrainStep: no collectives), the SH record
    all-gather alone and the flat all-reduce of the other four gradients alone, and reports
    the bytes each rank moves.  hidden_frac = 1 - (t_step - t_compute) / (t_allgather +
    t_allreduce): the share of the collectives' time that overlapped compute."""
    n = scene.num_points
    solo = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")

    def compute_only():
        solo.zero_grad()
        solo.forward_backward(cam, gt, bg)
    for _ in range(3):
        compute_only()
    t_comp = timed(compute_only, steps) / steps * 1e3
    rlen = record_floats or 3 * n + 4  # the record the step sent (sparse or dense)
    rec = torch.zeros(rlen, device=dev)
    gathered = torch.empty(world * rlen, device=dev)
    flat = torch.zeros(11 * n, device=dev)  # means 3 + scales 3 + quats 4 + opacity 1 floats
    for _ in range(3):
        dist.all_gather_into_tensor(gathered, rec)
        dist.all_reduce(flat)
    t_ag = timed(lambda: dist.all_gather_into_tensor(gathered, rec), steps) / steps * 1e3
    t_ar = timed(lambda: dist.all_reduce(flat), steps) / steps * 1e3
    for p in scene.params():
        p.grad = None
    return {
        "t_compute_only_ms": round(t_comp, 4),
        "t_allgather_ms": round(t_ag, 4),
        "t_allreduce_ms": round(t_ar, 4),
        "record": "dense" if rlen == 3 * n + 4 else "sparse",
        "bytes_allgather_recv_per_rank": (world - 1) * rlen * 4,
        "bytes_allreduce_per_rank": int(2 * (world - 1) / world * 11 * n * 4),  # ring send+recv
        "collectives_per_step": 2,
    }


def train_roofline(train_step, steps, barrier, ab, N, I, P, T, K, world, trainer, iters_per_s):
    """The train step's byte split (render vs loss vs Adam vs the exchange) and
    its time split, measured with HIP events around every C-ABI call over `steps` train steps
    (the step is re-run for this; the timed train_iters_per_s loop runs without events).
    Bytes: the render's §8d fwd+bwd model, the loss kernels' 132 P, Adam 24 B per parameter
    inside the fused backward (one GPU) or 28 B standalone (gsplat_adam_step), the exchange
    kernels' records; link bytes (N > 1) apart: per rank, the record all-gather receives
    (N - 1) records and the flat ring all-reduce moves 2 (N - 1) / N x 44 B per Gaussian."""
    if steps <= 0:
        return None
    with timing.timed_calls() as tm:
        barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(steps):
            train_step()
        ev1.record()
        calls = tm.summary()
        step_ms_events = ev0.elapsed_time(ev1) / steps
    params = (11 + 3 * K) * N
    if world > 1:  # the multi-view table kernels over R = world x views records (12 B each)
        R = world * getattr(trainer.sh_exchange, "views_per_step", 1) if trainer.sh_exchange \
            else world
        ab = dict(ab)
        ab["gsplat_compute_sh_backward_view_table"] = (12 + 12 * R + 12 * K) * N
        ab["gsplat_compute_sh_backward_view_table_adam"] = (12 + 12 * R + 24 * 3 * K) * N
        # the record packing: gradient record (64 B), radii and colours in, 12 B out (dense; a
        # sparse record writes only the visible rows); the visibility plan reads radii
        ab["gsplat_exchange_pack_colors"] = 92 * N
        ab["gsplat_exchange_pack_sparse"] = 92 * N
        ab["gsplat_exchange_sparse_plan"] = 4 * N
        if getattr(trainer, "fuse_sh_adam", False):  # the standalone Adam: geometry groups only
            ab["gsplat_adam_step"] = 28 * 11 * N
    render_bytes = (388 + 24 * K) * N + 124 * I + 44 * P + 8 * T
    parts_ms, parts_bytes = {}, {"render": render_bytes}
    for name, (ncalls, mean_ms, tot_ms) in calls.items():
        if "(side stream)" in name:
            continue  # (overlaps the step's own stream)
        part = train_part(name)
        parts_ms[part] = parts_ms.get(part, 0.0) + tot_ms / steps
        if part != "render":
            parts_bytes[part] = parts_bytes.get(part, 0) + int(ab.get(name, 0) * ncalls / steps)
    if "geometry backward + adam (one kernel)" in parts_bytes:
        # the render model counts the geometry backward's gradient traffic; the fused kernel's
        # bytes beyond it are the Adam update's (24 B per parameter)
        parts_bytes.pop("geometry backward + adam (one kernel)")
        parts_bytes["adam (inside the geometry backward)"] = 24 * params
    attributed = sum(parts_ms.values())
    step_ms = 1e3 / iters_per_s
    # the uninstrumented step minus the entries (see the bench line's kernels_timing: the event
    # records themselves add device time between the calls)
    parts_ms["(outside the C-ABI calls)"] = max(0.0, step_ms - attributed)
    hbm = sum(parts_bytes.values())
    out = {
        "step_ms": round(step_ms, 4),
        "step_ms_events": round(step_ms_events, 4),
        "time_ms_per_step": {k: round(v, 4) for k, v in parts_ms.items()},
        "algorithmic_bytes_per_step": parts_bytes,
        "algorithmic_bytes_total": hbm,
        "frac": round(hbm / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "adam_bytes_per_gaussian": 28 * (11 + 3 * K),
    }
    if world > 1:
        xc = trainer.sh_exchange
        rec = xc.last_record_floats if xc is not None and xc.last_record_floats else 3 * N
        out["link_bytes_per_rank"] = {
            "record_all_gather_in": 4 * rec * (world - 1),
            "geometry_all_reduce": int(2 * (world - 1) / world * 44 * N),
        }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--train-steps", type=int, default=None)
    ap.add_argument("--no-lane-occupancy", action="store_true",
                    help="skip the counted extra step (profiler runs: keeps the counting "
                         "kernels out of the PMC and kernel-trace summaries)")
    ap.add_argument("--forward-only", action="store_true",
                    help="time the render without backward (default for config c2)")
    ap.add_argument("--views-per-gpu", type=int, default=1,
                    help="views each rank renders per step (gradients summed over all; N > 1: "
                         "the record all-gathers of a rank's earlier views overlap its later "
                         "views, exchange.py)")
    ap.add_argument("--render", default="fused", choices=("fused", "caller"),
                    help="fused: the caller's activations inside the HIP kernels (default); "
                         "caller: gc_model.py's torch glue around the gsplat API")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank (RCCL); BENCH_DIST_BACKEND=gloo lets a one-GPU box rehearse the N > 1
    # path with every rank on its one device (ranks share it; not a scaling measurement)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local_rank %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    N, W, H, deg, lo, hi, seed, real, desc = CONFIGS[args.config]
    K = num_sh_bases(deg)
    scene, cam_cpu = make_workload(args.config, rank, dev)
    cam = cam_cpu.to(dev)
    H, W = cam.height, cam.width
    g = torch.Generator().manual_seed(1000 + rank)
    gt = torch.rand(H, W, 3, generator=g).to(dev)
    bg = torch.zeros(3, device=dev)
    trainer = TrainStep(scene, sh_degree=deg, world_size=world, loss="l1",
                        render_mode=args.render)
    caller = TrainStep(scene, sh_degree=deg, world_size=world, loss="l1", render_mode="caller")

    fwd_only = args.forward_only or args.config in FORWARD_ONLY

    V = max(args.views_per_gpu, 1)
    # several views per rank: rank r renders views r, r + N, r + 2N, ... of the config's set
    extra = [config_camera(args.config, rank + k * world).to(dev) for k in range(1, V)]
    gts = [gt] + [torch.rand(H, W, 3, generator=g).to(dev) for _ in range(1, V)]

    def step_views(t, cams):
        t.zero_grad()
        t.forward_backward_views(cams, gts[:len(cams)], bg)
        t.sync_grads()

    def step_eager(t=trainer, c=None):
        c = cam if c is None else c
        if V > 1 and not fwd_only and t.render_mode == "fused":
            step_views(t, [c] + extra)
            return
        if fwd_only:
            with torch.no_grad():
                if t.render_mode == "fused":
                    render_fused(scene, c, deg, bg)
                else:
                    render(scene, c, deg, bg)
            return
        t.zero_grad()
        t.forward_backward(c, gt, bg)
        t.sync_grads()

    step = step_eager

    def timed(fn, steps):
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # settle: a fixed number of untimed steps before anything is timed, so that every leg
    # starts at the GPU's steady-state clocks -- with the driver's --steps 20 --warmup 5 and
    # the caller leg alone in front, the headline still read 1,567-1,568 against 1,604 at
    # steady state (profiles/r06_warmup_sensitivity.txt).  A step count, not a time, so every
    # rank runs the same collectives at N > 1.
    for _ in range(SETTLE_STEPS):
        step()
    barrier()
    # the same step through the unchanged caller's torch glue (gc_model.py as it runs on the
    # gsplat drop-in), for comparison
    for _ in range(max(args.warmup // 2, 1)):
        step(caller)
    caller_value = world * H * W * args.steps / timed(lambda: step(caller), args.steps) / 1e6

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    value = world * V * H * W * args.steps / dt / 1e6
    value_2v = None
    if world > 1 and V == 1 and not fwd_only and args.render == "fused":
        # the same job with two views per rank per step (exchange.py: the first view's record
        # all-gather overlaps the second view's render): the step's per-view throughput
        cams2 = [cam, config_camera(args.config, rank + world).to(dev)]
        gts2 = [gt, torch.rand(H, W, 3, generator=torch.Generator().manual_seed(77 + rank)).to(dev)]

        def two():
            trainer.zero_grad()
            trainer.forward_backward_views(cams2, gts2, bg)
            trainer.sync_grads()
        for _ in range(3):
            two()
        value_2v = round(world * 2 * H * W * args.steps / timed(two, args.steps) / 1e6, 2)
    rotating = rotating_cameras(args.config, rank, dev, step_eager, timed, args.steps,
                                world * V)
    exch = None
    if world > 1 and not fwd_only:
        xc = trainer.sh_exchange
        exch = exchange_profile(scene, cam, gt, bg, deg, world, dev, args.steps, timed,
                                xc.last_record_floats if xc is not None else None)
        comm = exch["t_allgather_ms"] + exch["t_allreduce_ms"]
        exch["t_step_ms"] = round(ms_per_step, 4)
        exch["exposed_ms"] = round(ms_per_step - exch["t_compute_only_ms"], 4)
        exch["hidden_frac"] = round(1 - exch["exposed_ms"] / comm, 3) if comm > 0 else None
        exch["backend"] = backend
    # per-entry-point device time (HIP events on the launch stream), same step, K steps
    with timing.timed_calls() as tm:
        barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(args.steps):
            step_eager()
        ev1.record()
        per_call = tm.summary()
        events_step_ms = ev0.elapsed_time(ev1) / args.steps
    with torch.no_grad():
        from gaussctrl_exp_amd.project_gaussians import project_gaussians
        xys, depths, radii, conics, nth, _ = project_gaussians(
            scene.means, torch.exp(scene.scales), 1,
            scene.quats / scene.quats.norm(dim=-1, keepdim=True), *cam.project_args())
        I, _, _ = bin_gaussians(xys, depths, radii, nth, H, W)
        nvis = int((radii > 0).sum().item())
    T = cam.tile_bounds[0] * cam.tile_bounds[1]
    P = H * W
    ab = algorithmic_bytes(N, I, P, T, K, nvis)
    kernels = {}
    for name, (calls, mean_ms, tot_ms) in per_call.items():
        per_step = calls / args.steps
        b = ab.get(name)
        hb = pmc_traffic(name, args.config)
        kernels[name] = {
            "ms_per_call": round(mean_ms, 4),
            "calls_per_step": per_step,
            # algorithmic bytes (SURVEY.md §8d model) / time: bytes the L2 / MALL serve count
            # too, so this can exceed the 8 TB/s HBM peak (c5's forward); hbm_GBps is the
            # rocprofv3 PMC HBM traffic (FETCH_SIZE + WRITE_SIZE, profiles/pmc_traffic.json) of
            # this config / time, null without counters
            "alg_bytes": b,
            "alg_GBps": round(b / (mean_ms * 1e-3) / 1e9, 1) if b else None,
            "hbm_bytes": hb,
            "hbm_GBps": round(hb / (mean_ms * 1e-3) / 1e9, 1) if hb else None,
        }
    # the entries' device time per step against the uninstrumented step (ms_per_step): the
    # remainder is torch work outside the C ABI (loss glue, zero_grad, all-reduce) and device
    # idle between calls, so the block sums to the step.  The instrumented loop runs longer
    # (step_ms_events; headline ~0.05 ms per step for its 14 event records, each a packet with
    # its own completion signal), and that time lands between the calls -- counted apart, as
    # instrumentation_ms_per_step, not as the step's own idle.
    # (entries on a second stream overlap the others: not part of the sum)
    attributed = sum(v[2] for k, v in per_call.items() if "(side stream)" not in k) / args.steps
    kernels["(outside the C-ABI calls)"] = {
        "ms_per_call": round(max(0.0, ms_per_step - attributed), 4), "calls_per_step": 1.0,
        "alg_bytes": None, "alg_GBps": None, "hbm_bytes": None, "hbm_GBps": None}
    kernels_timing = {
        "method": "HIP events recorded on the launch stream before and after each C-ABI call "
                  "(device timestamps; an entry's time includes device idle while the host "
                  "issues that call's launches); outside = ms_per_step - sum of the entries",
        "step_ms_events": round(events_step_ms, 4),
        "instrumentation_ms_per_step": round(events_step_ms - ms_per_step, 4),
        "sum_entries_ms_per_step": round(attributed, 4),
    }
    step_hbm = 0
    for name, (calls, mean_ms, tot_ms) in per_call.items():
        hb = kernels[name]["hbm_bytes"]
        if hb is None:
            step_hbm = None
            break
        step_hbm += int(hb * calls / args.steps)
    dom = max(per_call, key=lambda k: per_call[k][2])
    dom_ms = per_call[dom][1]
    dom_bytes = ab.get(dom)
    # the step's algorithmic bytes per view: SURVEY.md §8d's model (the per-entry models above
    # count every radix pass; this one counts the binning as gsplat's map + one sort + bins)
    step_bytes = (124 * N + 84 * I + 20 * P + 8 * T) if fwd_only else \
        ((388 + 24 * K) * N + 124 * I + 44 * P + 8 * T)
    roofline = {
        "kernel": dom,
        "bound": "hbm",
        "achieved": round(dom_bytes / (dom_ms * 1e-3) / 1e9, 1) if dom_bytes else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if dom_bytes else None,
        "traffic": pmc_traffic(dom, args.config),
        "traffic_fetch_scale": 2 if ENTRY_KERNELS.get(dom, ((), False))[1] else 1,
        "valu_busy": pmc_valu_busy(dom, args.config, dom_ms),
        "valu_issue_frac": pmc_issue_and_wait(dom, args.config, dom_ms)[0],
        "wait_frac": pmc_issue_and_wait(dom, args.config, dom_ms)[1],
        "issue_stall_frac": pmc_issue_and_wait(dom, args.config, dom_ms)[2],
        "step_algorithmic_bytes": step_bytes,
        "step_frac": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        # the step's HBM bytes as the PMC counters saw them (sum over the entries on the step's
        # stream of hbm_bytes x calls; null when an entry has no counters for this config)
        "step_hbm_bytes_pmc": step_hbm,
        "step_hbm_frac_pmc": (round(step_hbm / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                              if step_hbm else None),
        "roofline_mpix_s": round(P / (step_bytes / (HBM_PEAK_GBS * 1e9)) / 1e6, 1),
    }

    lanes = None if args.no_lane_occupancy else lane_occupancy(step_eager, dev, args.config)

    # full train step: splatfacto loss + backward + all-reduce + Adam
    tsteps = args.train_steps if args.train_steps is not None else args.steps
    trainer.loss_kind = "splatfacto"

    def train_step():
        trainer.step(cam, gt)

    def train_time(fn):
        for _ in range(2):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(tsteps):
            fn()
        barrier()
        tdt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([tdt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tdt = float(t.item())
        return tdt
    tdt = train_time(train_step)
    train_rl = train_roofline(train_step, tsteps, barrier, ab, N, I, P, T, K, world,
                              trainer, tsteps / tdt)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scene, cam_cpu, deg, backward=not fwd_only)

    if rank == 0:
        line = {
            "metric": ("Mpixels/s fwd+bwd and train iters/s, 1M Gaussians @ 1080^2"
                       if not fwd_only else "Mpixels/s forward and train iters/s"),
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": SETTLE_STEPS,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": ("synthetic (random-Gaussian scene per SURVEY.md §8d; random-init params)"
                     if real is None else f"{real} cameras + seed cloud (tests/golden); "
                     "random-init Gaussians around the seeds; synthetic GT"),
            "config": {
                "workload": desc,
                "num_gaussians": N,
                "num_visible": nvis,
                "num_intersects": I,
                "tiles": T,
                "image": [H, W],
                "sh_degree": deg,
                "views_per_gpu_per_step": V,
                "parallelism": f"dp{world} ({V} view/GPU; SH-coefficient grads by RCCL "
                               f"all-gather of each view's colour-gradient record (sparse: "
                               f"visible Gaussians only, when smaller) + multi-view SH backward, "
                               f"other {N * 11 * 4} B of grads RCCL all-reduced)" if world > 1
                               else "dp1",
            },
            "render": args.render,
            "exchange": exch,
            "value_2_views_per_gpu": value_2v,
            "value_rotating_cameras": rotating["value"],
            "speculative_misses": rotating["misses"],
            "rotating_cameras": rotating["desc"],
            "value_unchanged_caller": round(caller_value, 2),
            "train_iters_per_s": round(tsteps / tdt, 2),
            "train_views_per_s": round(world * tsteps / tdt, 2),
            "roofline": roofline,
            "train_roofline": train_rl,
            "lane_occupancy": lanes,
            "kernels": kernels,
            "kernels_timing": kernels_timing,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
