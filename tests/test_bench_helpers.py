"""bench.py's CPU-side helpers: the critical-path bound it reports beside the VALU roofline, and
the PMC files it reads (`roofline.traffic`, the full batch's write ratio), which must match the
kernel the bench times or be reported as absent."""
import json
import os

import pytest

import bench


def test_critical_path_model():
    # the headline: 100k columns, 391 strips of 256 rows, 9 VALU per step at 4 cycles, 2.4 GHz
    cp = bench.critical_path(100000, 391, 9, 5.5, 256)
    assert cp["steps"] == 100000 + 391 * 64
    assert cp["step_cycles_bound"] == 36
    assert cp["bound_ms"] == pytest.approx(125024 * 36 / 2.4e9 * 1e3, rel=1e-4)
    assert cp["frac"] == pytest.approx(cp["bound_ms"] / 5.5, rel=1e-3)
    assert cp["step_cycles_achieved"] == pytest.approx(5.5e-3 * 2.4e9 / 125024, rel=1e-3)


def test_traffic_file_matches_the_bench_kernel():
    """profiles/traffic_config3.json is read into roofline.traffic only for the kernel, R and C the
    bench runs: the committed file must name the current headline kernel."""
    p = os.path.join(bench.ROOT, "profiles", "traffic_config3.json")
    tj = json.load(open(p))
    kname = bench.sparse_kernel_name()
    assert tj["kernel"] == kname
    assert bench.traffic_for("traffic_config3.json", tj["R"], tj["C"], kname) == tj["hbm_bytes_per_launch"]
    assert bench.traffic_for("traffic_config3.json", tj["R"], tj["C"], "another kernel") is None
    assert bench.traffic_for("no_such_file.json", tj["R"], tj["C"], kname) is None
    # the PMC bytes are the headers written plus the granules written and read once
    alg = tj["algorithmic_bytes"]
    assert tj["hbm_bytes_per_launch"] == pytest.approx(sum(alg.values()), rel=0.05)


def test_full_batch_write_ratio(monkeypatch):
    """The full_batch field's PMC write ratio comes from the round-4 profile of the kernels the
    batch runs by default (the two-pass fill in two launches), and only for them."""
    for k in ("GSA_FULL_KERNEL", "GSA_FULL_FUSED"):
        monkeypatch.delenv(k, raising=False)
    r = bench.pmc_write_ratio(64, bench.full_kernel_name(False))
    assert r is not None and 1.0 <= r <= 1.05
    assert bench.pmc_write_ratio(32, bench.full_kernel_name(False)) is None
    assert bench.pmc_write_ratio(64, "gsa::nw_lane_kernel<4,false,true>") is None


def test_rehearsal_fields(monkeypatch):
    """A GSA_BENCH_REHEARSE run (N gloo ranks sharing cuda:0) reports one GPU and says it is a
    rehearsal, so its line can never pass as a multi-GPU result; a real run reports its ranks."""
    monkeypatch.setattr(bench, "REHEARSE", True)
    f = bench.gpu_fields(2)
    assert f["n_gpus"] == 1 and f["rehearsal"] is True and "REHEARSAL" in f["parallelism"]
    monkeypatch.setattr(bench, "REHEARSE", False)
    f = bench.gpu_fields(8)
    assert f == {"n_gpus": 8, "rehearsal": False, "parallelism": "pair-sharded x8"}


def test_score_kernel_label(monkeypatch):
    """The config5 field names the kernel that gsa_score_dev runs (K-rows by default,
    the strip kernel under GSA_SCORE_KERNEL=strip)."""
    monkeypatch.delenv("GSA_SCORE_KERNEL", raising=False)
    monkeypatch.delenv("GSA_KROW_Q8", raising=False)
    monkeypatch.delenv("GSA_SCORE_K", raising=False)
    monkeypatch.delenv("GSA_SCORE_BIDI", raising=False)
    monkeypatch.delenv("GSA_SCORE_BIDI_SW", raising=False)
    assert bench.score_kernel_name(-11, -1, False).startswith("gsa::nw_kscore_kernel<3, false, 2>")
    assert bench.score_kernel_name(-11, -11, True).startswith("gsa::nw_kscore_kernel<5, false, 2>")
    # NW at 50k: both ends at 2 rows per lane; one direction for an odd R or a short pair
    assert "both ends" in bench.score_kernel_name(-11, -1, False)
    assert bench.score_kernel_name(-11, -11, False).startswith("gsa::nw_kscore_kernel<6, false, 2> (kModeScoreAGL, both")
    assert "both ends" in bench.score_kernel_name(-11, -11, False, R=49999)  # transposed
    assert bench.score_kernel_name(-11, -11, False, R=49999, C=49999).startswith("gsa::nw_kscore_kernel<6, true, 4>")
    assert bench.score_kernel_name(-11, -11, False, R=4000, C=4000).startswith("gsa::nw_kscore_kernel<6, true, 4>")
    # SW: by rows only (three pairs), one direction for an odd R or under GSA_SCORE_BIDI_SW=0
    assert "bottom fresh" in bench.score_kernel_name(-11, -11, True)
    assert "both ends" not in bench.score_kernel_name(-11, -11, True, R=49999)
    monkeypatch.setenv("GSA_SCORE_BIDI_SW", "0")
    assert "both ends" not in bench.score_kernel_name(-11, -11, True)
    monkeypatch.delenv("GSA_SCORE_BIDI_SW")
    monkeypatch.setenv("GSA_SCORE_BIDI", "0")
    assert bench.score_kernel_name(-11, -11, False).startswith("gsa::nw_kscore_kernel<6, true, 4>")
    monkeypatch.delenv("GSA_SCORE_BIDI")
    monkeypatch.setenv("GSA_SCORE_KERNEL", "strip")
    assert "nw_strip_kernel" in bench.score_kernel_name(-11, -1, False)


def test_full_kernel_label(monkeypatch):
    """The 10k and full_batch fields name the kernels gsa_capi.hip's full-fill routing runs: the fused
    single-pair kernel by default, the two launches under GSA_FULL_FUSED=0 and for batches, the lane
    fill under GSA_FULL_KERNEL=lane."""
    for k in ("GSA_FULL_KERNEL", "GSA_FULL_FUSED", "GSA_LANE_NS", "GSA_LANE_FEED", "GSA_LANE_PAIR"):
        monkeypatch.delenv(k, raising=False)
    assert bench.full_kernel_name(True).startswith("gsa::nw_full_fused_kernel<4,8,true,3>")
    assert bench.full_kernel_name(False).startswith("gsa::nw_krow_kernel<8,4,1024,2,true>")
    monkeypatch.setenv("GSA_FULL_FUSED", "0")
    assert bench.full_kernel_name(True).startswith("gsa::nw_krow_kernel<4,4,1024,2,true>")
    monkeypatch.setenv("GSA_FULL_KERNEL", "lane")
    assert bench.full_kernel_name(True).startswith("gsa::nw_lane_kernel<4,true,false>")
    monkeypatch.setenv("GSA_FULL_KERNEL", "twopass")
    assert "nw_expand_stream_kernel" in bench.full_kernel_name(False)


def test_pass_fields_out_fill():
    """full_batch.passes: pass 2's rate beside the runtime fill kernel's over the same output buffer."""
    tm = {"pass1_ms": 4.0, "pass2_ms": 20.0, "out_fill_ms": 16.0, "out_fill_bytes": 110 * 10**9}
    f = bench.pass_fields(tm, 100e9)
    assert f["pass2_write_GBps"] == 5000.0 and f["out_fill_GBps"] == 6875.0
    assert f["pass2_over_out_fill"] == round(5000.0 / 6875.0, 4)
    assert f["pass1_share"] == round(4 / 24, 4)
    assert "out_fill_ms" not in bench.pass_fields({"pass1_ms": 1.0, "pass2_ms": 2.0}, 1e9)
