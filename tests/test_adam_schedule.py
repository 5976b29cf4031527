"""The device schedule of the in-backward Adam step (optim.adam_schedule_table, read by
gsplat_fused_preprocess_backward_adam_sched): every entry equals what the host path passes the
kernel (gsplat_fused_preprocess_backward_adam: float(lr) and float betas into C double pow /
division / sqrt, rounded to float), and the last row stands for every later step -- the table's
clamp is exact.  CPU only (the GPU equality of the two kernels: tests/test_gpu_graphs.py)."""
import math

import numpy as np

from gaussctrl_exp_amd.optim import adam_schedule_table
from gaussctrl_exp_amd.scene import synthetic_scene
from gaussctrl_exp_amd.train import XYZ_MAX_STEPS, TrainStep

BETAS = (0.9, 0.999)


def _host(lrs, c):
    """The values gsplat_fused_preprocess_backward_adam computes for step t = c + 1."""
    b1, b2 = float(np.float32(BETAS[0])), float(np.float32(BETAS[1]))
    t = c + 1
    bc1, bc2 = 1.0 - math.pow(b1, t), 1.0 - math.pow(b2, t)
    ss = [np.float32(float(np.float32(lr)) / bc1) for lr in lrs]
    return ss, np.float32(math.sqrt(bc2))


def test_table_matches_the_host_schedule():
    tr = TrainStep(synthetic_scene(8, 3, seed=1), sh_degree=3, render_mode="caller")
    table = adam_schedule_table(tr._lrs_of_step, BETAS, XYZ_MAX_STEPS + 1)
    assert table.shape == (7, XYZ_MAX_STEPS + 1) and table.dtype == np.float32
    for c in (0, 1, 2, 9, 99, 1000, 17000, 29999, XYZ_MAX_STEPS):
        ss, bc2s = _host(tr._lrs_of_step(c), c)
        for k in range(6):
            assert table[k, c] == ss[k], (c, k)
        assert table[6, c] == bc2s, c
    # means decays (splatfacto's exponential schedule), the rest stays
    assert table[0, 0] > table[0, 15000] > table[0, XYZ_MAX_STEPS]
    assert table[4, 5000] == table[4, XYZ_MAX_STEPS]


def test_last_row_stands_for_every_later_step():
    tr = TrainStep(synthetic_scene(8, 3, seed=1), sh_degree=3, render_mode="caller")
    table = adam_schedule_table(tr._lrs_of_step, BETAS, XYZ_MAX_STEPS + 1)
    for c in (XYZ_MAX_STEPS + 1, 40000, 10 ** 6):
        ss, bc2s = _host(tr._lrs_of_step(c), c)
        for k in range(6):
            assert table[k, -1] == ss[k], (c, k)
        assert table[6, -1] == bc2s, c
