"""Check the one-sweep radix sort (gsplat_sort_isect_pairs) against numpy's stable sort."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from gaussctrl_exp_amd import _lib

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
HEAD_ERR_OFF = (8 * 256 + 8) * 4
for n, bits, hi in [(100, 13, 4624), (4096, 13, 4624), (4097, 13, 4624), (20000, 13, 4624),
                    (20000, 41, 1 << 41), (100000, 13, 4624), (100000, 32, 1 << 32),
                    (1000000, 32, 1 << 32), (8000000, 13, 4624)]:
    keys = rng.integers(0, hi, size=n, dtype=np.int64)
    vals = np.arange(n, dtype=np.int32)
    k = torch.from_numpy(keys).to(dev)
    v = torch.from_numpy(vals).to(dev)
    ko, vo = torch.empty_like(k), torch.empty_like(v)
    wsz = _lib.query("gsplat_sort_isect_pairs_workspace_size", n)
    ws = torch.zeros(wsz, dtype=torch.uint8, device=dev)
    P = _lib.ptr
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _lib.call("gsplat_sort_isect_pairs", n, bits, P(k), P(v), P(ko), P(vo), P(ws), wsz,
              _lib.stream(dev))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # radix workspace begins after 2 key + 2 val buffers (256-B aligned)
    al = lambda x: (x + 255) // 256 * 256
    rs_off = 2 * al(n * 8) + 2 * al(n * 4)
    err = int(ws[rs_off + HEAD_ERR_OFF: rs_off + HEAD_ERR_OFF + 4].cpu().view(torch.int32)[0])
    order = np.argsort(keys, kind="stable")
    ok_k = np.array_equal(ko.cpu().numpy(), keys[order])
    ok_v = np.array_equal(vo.cpu().numpy(), vals[order])
    bad = np.nonzero(ko.cpu().numpy() != keys[order])[0]
    print(f"n={n:8d} bits={bits:2d} keys_ok={ok_k} vals_ok={ok_v} err={err} "
          f"bad={len(bad)} first_bad={bad[:5].tolist()} ms={dt*1e3:.2f}", flush=True)
