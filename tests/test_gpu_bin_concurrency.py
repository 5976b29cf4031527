"""bin_gaussians calls in flight at once on different streams and host threads: each call
polls its own pinned count slot (rasterize._CountSlots), so a queued scan of one call never
overwrites the intersection count another call is waiting for."""
import threading

import numpy as np
import pytest
import torch

import oracle as O
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

pytestmark = pytest.mark.gpu


def _scene(gpu, n, seed, W, H):
    sc = synthetic_scene(n, 0, seed=seed, scale_lo=0.005, scale_hi=0.03).to(gpu)
    cam = synthetic_camera(W, H).to(gpu)
    with torch.no_grad():
        g = project_gaussians(sc.means, torch.exp(sc.scales), 1,
                              sc.quats / sc.quats.norm(dim=-1, keepdim=True),
                              *cam.project_args())
    return [t.detach() for t in g], cam


def test_two_streams_two_threads_bin_concurrently(gpu, oracle_lib):
    scenes = [_scene(gpu, 200_000, 1, 1024, 768), _scene(gpu, 30_000, 2, 320, 256)]
    refs = []
    for (xys, depths, radii, conics, nth, _), cam in scenes:
        r = O.bin_and_sort(xys.cpu().numpy(), depths.cpu().numpy(), radii.cpu().numpy(),
                           nth.cpu().numpy(), cam.tile_bounds)
        refs.append(r)
    assert refs[0]["num_intersects"] != refs[1]["num_intersects"]
    torch.cuda.synchronize()
    results = [[] for _ in scenes]
    errors = []
    start = threading.Barrier(len(scenes))

    def worker(k):
        try:
            (xys, depths, radii, conics, nth, _), cam = scenes[k]
            s = torch.cuda.Stream(gpu)
            with torch.cuda.stream(s):
                start.wait()
                for _ in range(12):
                    I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
                    results[k].append((I, gids, bins))
            s.synchronize()
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(len(scenes))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    for k, ref in enumerate(refs):
        assert len(results[k]) == 12
        for I, gids, bins in results[k]:
            assert I == ref["num_intersects"]
        I, gids, bins = results[k][-1]
        np.testing.assert_array_equal(gids.cpu().numpy(), ref["gaussian_ids_sorted"])
        np.testing.assert_array_equal(bins.cpu().numpy(), ref["tile_bins"])
