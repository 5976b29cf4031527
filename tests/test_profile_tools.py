"""Counter attribution of the profile tools and bench.py: kernel rows are keyed by the full
template instantiation, and an entry's per-step figures come from the instantiation its timed
step launched (the most-dispatched one), not a sum over every instantiation that ran."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

from kname import short_name  # noqa: E402
import bench  # noqa: E402


def test_instantiations_keep_distinct_keys():
    a = "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(4)>(float const*, int)"
    b = "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(2)>(float const*, int)"
    assert short_name(a) != short_name(b)
    assert short_name(a).endswith("float __vector(4)>")
    assert short_name("gs::(anonymous namespace)::k<3>(int)") == "gs::k<3>"
    assert short_name("__amd_rocclr_fillBufferAligned") == "__amd_rocclr_fillBufferAligned"


def test_entry_uses_the_step_instantiation(monkeypatch):
    kern = {
        "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(4)>":
            {"insts_valu": 100.0, "fetch_kb": 10.0, "write_kb": 1.0, "dispatches": 52},
        "void gs::raster_bwd3p_kernel<1, true, 16, false, float __vector(4)>":
            {"insts_valu": 900.0, "fetch_kb": 90.0, "write_kb": 9.0, "dispatches": 3},
    }
    monkeypatch.setattr(bench, "_pmc_kernels", lambda config: kern)
    monkeypatch.setattr(bench, "_pmc_entry", lambda entry, config: None)
    assert bench.pmc_insts_valu("gsplat_rasterize_backward_records_l1", "headline") == 100.0
    assert bench.pmc_traffic("gsplat_rasterize_backward_records_l1", "headline") == 11 * 1024
    # an entry with two kernels takes one instantiation of each
    kern["void gs::split_grads_kernel"] = {"insts_valu": 5.0, "dispatches": 52}
    assert bench.pmc_insts_valu("gsplat_rasterize_backward", "headline") == 105.0


def test_entry_pattern_parts_select_the_adam_instantiation(monkeypatch):
    """'&'-separated pattern parts must all match: the in-backward Adam entry takes the
    <K, true> fused backward, the plain one the <K, false> one, even when the other is
    dispatched more often."""
    kern = {
        "void gs::fused_bwd_kernel<16, false>": {"fetch_kb": 1.0, "write_kb": 0.0, "dispatches": 80},
        "void gs::fused_bwd_kernel<16, true>": {"fetch_kb": 7.0, "write_kb": 0.0, "dispatches": 7},
    }
    monkeypatch.setattr(bench, "_pmc_kernels", lambda config: kern)
    monkeypatch.setattr(bench, "_pmc_entry", lambda entry, config: None)
    # (streaming kernels: FETCH_SIZE x 2, MI355X_MICROARCH.md)
    assert bench.pmc_traffic("gsplat_fused_preprocess_backward", "headline") == 2 * 1024
    assert bench.pmc_traffic("gsplat_fused_preprocess_backward_adam", "headline") == 14 * 1024


def test_train_parts():
    assert bench.train_part("gsplat_l1_ssim_forward") == "loss"
    assert bench.train_part("gsplat_adam_step") == "adam"
    assert bench.train_part("gsplat_compute_sh_backward_view_table_adam").startswith("exchange")
    assert bench.train_part("gsplat_exchange_pack_sparse").startswith("exchange")
    assert bench.train_part("gsplat_bin_speculative") == "render"
    assert bench.train_part("gsplat_fused_preprocess_backward_adam").startswith("geometry")
