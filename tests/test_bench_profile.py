"""The committed PMC profile that bench.py reads `roofline.traffic` and
`measured_GBps` from (profiles/*traffic*.json): it must be
a profile of the current HIP sources, and it must hold every kernel symbol the
default bench run looks up, or the bench line silently reports null."""
import pytest

import bench

CELLS_512 = float(510 ** 3)


def test_profile_is_current_and_complete():
    prof = bench.pmc_profile(CELLS_512)
    if prof is None:
        pytest.xfail("no PMC profile of the current cfd_amd/csrc/hip sources: "
                     "re-run tools/gpu_profile.sh and commit its traffic.json")
    # the default run: 1 rank at 512^3, 16-row sweeps, variant 15, the CG
    # variant bench.cg_variant_auto picks there (single-reduction)
    variant = bench.cg_variant_auto(512, 1)
    assert variant == 1
    want = [k for _, k, _ in bench.sweep_kernels(16, False, 15, variant)]
    want += list(bench.TIMER_KERNEL.values())
    recs = {k: bench.prof_record(prof, k) or {} for k in want}
    missing = [k for k, r in recs.items() if "hbm_bytes_per_launch" not in r]
    assert not missing, missing
    for k in want:
        assert recs[k]["hbm_bytes_per_launch"] > 0


def test_cg_variant_auto_and_fused_record(monkeypatch):
    # single-reduction where it is measured faster: one GPU at 512^3; on
    # Z-slabs the variant the committed slab budget projects faster at that
    # N, textbook CG where it has no projection
    assert bench.cg_variant_auto(512, 1) == 1
    assert bench.cg_variant_auto(256, 1) == 0
    assert bench.cg_variant_auto(512, 1, "tg") == 0
    assert bench.cg_variant_auto(512, 8, "tg") == 0
    budget = {"projected_ms_per_iter": {"2": {"cg0": 0.70, "cg1": 0.65},
                                        "8": {"cg0": 0.20, "cg1": 0.21}}}
    monkeypatch.setattr(bench, "slab_budget", lambda: budget)
    assert bench.cg_variant_auto(512, 2) == 1
    assert bench.cg_variant_auto(512, 8) == 0
    assert bench.cg_variant_auto(512, 4) == 0  # no projection for N = 4
    assert bench.cg_variant_auto(256, 2) == 0  # the budget is of 512^3 slabs
    monkeypatch.setattr(bench, "slab_budget", lambda: None)
    assert all(bench.cg_variant_auto(512, w) == 0 for w in (2, 4, 8))
    # the fused timer's bytes: launch-weighted over k_ccf<*, *, false> only
    prof = {"kernels": {
        "k_ccf<true, false, false>": {"calls": 1, "hbm_bytes_per_launch": 10.0},
        "k_ccf<false, false, false>": {"calls": 5, "hbm_bytes_per_launch": 20.0},
        "k_ccf<false, true, false>": {"calls": 2, "hbm_bytes_per_launch": 50.0},
        "k_ccf<false, false, true>": {"calls": 9, "hbm_bytes_per_launch": 999.0}}}
    rec = bench.prof_record(prof, "k_ccf<false, false, false>")
    assert rec["hbm_bytes_per_launch"] == pytest.approx((10 + 100 + 100) / 8)
    assert bench.prof_record(prof, "k_ccf<false, false, true>")["hbm_bytes_per_launch"] == 999.0
    # per timer (ABI 3): the first + plain launches, and the fold launch alone
    rec = bench.prof_record(prof, "k_ccf<false, false, false>", "cc_fused")
    assert rec["hbm_bytes_per_launch"] == pytest.approx((10 + 100) / 6)
    rec = bench.prof_record(prof, "k_ccf<false, false, false>", "cc_fold")
    assert rec["hbm_bytes_per_launch"] == pytest.approx(50.0)


def test_ccf_split_and_committed_budget():
    kt = {"cc_fused": (30.0, 30), "cc_fold": (20.0, 10)}
    out = bench.ccf_split(kt, 1000, 1)
    assert out["cc_fused"]["avg_ms"] == 1.0 and out["cc_fold"]["avg_ms"] == 2.0
    assert out["cc_fused"]["bytes_per_cell"] == 32.0 and out["cc_fold"]["bytes_per_cell"] == 64.0
    assert bench.ccf_split({"cc_fused": (0.0, 0), "cc_fold": (0.0, 0)}, 10, 1)["cc_fold"] is None
    b = bench.slab_budget()
    if b is not None:  # a committed budget projects both variants at every N it covers
        for w, proj in b["projected_ms_per_iter"].items():
            assert int(w) > 1 and proj["cg0"] > 0 and proj["cg1"] > 0


def test_sweep_symbols_track_the_variant():
    one = dict((t, k) for t, k, _ in bench.sweep_kernels(16, True, 15, 0))
    assert one["cg_sweep_a"] == "k_cgA<16, false, true, 15, false>"
    assert one["cg_sweep_bx"] == "k_cgA<16, false, true, 11, true>"
    # cg_variant 1: one fused launch per iteration on one device (k_ccf); on
    # Z-slabs the march without its last stage + k_cc2 without the w store
    cc = dict((t, k) for t, k, _ in bench.sweep_kernels(16, False, 15, 1))
    assert cc == {"cc_march": "k_ccf<false, false, false>"}
    ccd = dict((t, k) for t, k, _ in bench.sweep_kernels(16, True, 15, 1, 64))
    assert ccd == {"cc_march": "k_ccf<false, false, false>",
                   "cc_spmv": "k_cc2<16, true, false, false>"}
    # the edge planes' k_cc2: 8 B per edge-plane cell, per slab cell 8 x 2 / planes
    assert dict((t, b) for t, _, b in bench.sweep_kernels(16, True, 15, 1, 64))["cc_spmv"] == 0.25


def test_cg_probe_rule():
    import argparse
    a = lambda probe, case="cavity": argparse.Namespace(cg_probe=probe, case=case)
    # default: N > 1, the bench's own choice, at the metric's 512^3 only
    assert bench.cg_probe_wanted(a("auto"), 512, 8, True)
    assert not bench.cg_probe_wanted(a("auto"), 512, 8, False)  # --cg-variant given
    assert not bench.cg_probe_wanted(a("auto"), 256, 8, True)
    assert not bench.cg_probe_wanted(a("auto"), 512, 1, True)   # one GPU: settled
    assert not bench.cg_probe_wanted(a("auto", "tg"), 512, 8, True)
    assert bench.cg_probe_wanted(a("on"), 66, 2, False)
    assert not bench.cg_probe_wanted(a("on"), 66, 1, True)
    assert not bench.cg_probe_wanted(a("off"), 512, 8, True)
    ch = bench.cg_variant_choice(2, a("auto"), {"picked": 1})
    assert ch["probe"] == {"picked": 1} and "live probe" in ch["rule"]
