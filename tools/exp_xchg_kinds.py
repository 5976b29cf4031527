"""Record kinds of the fused exchange over several steps (world 2, gloo, both ranks on one GPU):
per step each rank's (sparse, dense) counts, the agreed capacity and N.  Launch with
torch.distributed.run --nproc-per-node 2 tools/exp_xchg_kinds.py <config> <steps>."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gaussctrl_exp_amd.train import TrainStep  # noqa: E402


def main():
    cfg, steps = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    scene, cam = bench.make_workload(cfg, rank, dev)
    cam = cam.to(dev)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(rank)).to(dev)
    t = TrainStep(scene, sh_degree=3, world_size=world, loss="l1", render_mode="fused")
    bg = torch.zeros(3, device=dev)
    for s in range(steps):
        t.step(cam, gt, background=bg, optimizer=False)
        torch.cuda.synchronize()
        x = t.sh_exchange
        print(f"rank {rank} step {s}: kinds {x.record_kinds} cap {x.last_capacity} "
              f"n {scene.num_points} floats {x.last_record_floats}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
