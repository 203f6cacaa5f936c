"""CPU checks of bench.py's roofline bookkeeping (no GPU): the per-phase kernel parts of a
half-sweep, the counter lookup by workload / kernel / grid, the combination of several
kernels' counters in one launch-1 phase, and the top-k kernel / grid naming that
must match csrc/topk.hip's launch choice."""
import importlib.util
import os
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _block(n_light, n_chunks, n_short, n_short64):
    blk = SimpleNamespace(n_light=n_light, n_chunks=n_chunks)
    blk.n_dual = lambda rank: n_short if rank > 64 else (n_short64 if rank > 32 else 0)
    return blk


def test_launch1_parts_name_the_dual_kernel(bench):
    b = _block(1000, 10, 600, 200)
    assert bench._launch1_parts(b, 128, False) == [
        ("gram_solve_w1_kernel<false>", 64 * (10 + 400)), ("gram_solve_dual_kernel<128>", 64 * 600)]
    assert bench._launch1_parts(b, 64, False) == [
        ("gram_solve_kernel<4,false>", 64 * (10 + 800)), ("gram_solve_dual_kernel<64>", 64 * 200)]
    assert bench._launch1_parts(b, 128, True) == [("gram_solve_w1_kernel<true>", 64 * 1010)]
    assert bench._launch1_parts(b, 16, False) == [("gram_solve_kernel<1,false>", 64 * 1010)]
    assert bench._launch1_parts(b, 128, False, reg=0.0) == [("gram_solve_w1_kernel<false>", 64 * 1010)]


def test_bench_refuses_a_redirected_library(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, ALS_HIP_LIB=str(tmp_path / "libdev.so"))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-big"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "ALS_HIP_LIB" in p.stderr


def test_library_record_names_the_in_tree_build(bench):
    rec = bench.library_record()
    assert rec["path"].endswith("libals_hip.so") and not rec["path"].startswith("..")
    assert len(rec["sha256"]) == 64


def test_phase_counters_combine_by_grid(bench, monkeypatch):
    doc = {"format": 2, "workloads": {"w": {
        "gram_solve_w1_kernel<false>": {"by_grid": {"640": {
            "fetch_bytes_x2": 4e9, "write_bytes": 1e8, "pmc_run_avg_ns": 3e6, "trace_avg_ns": 3e6,
            "mfma_busy_frac": 0.4, "valu_busy_frac": 0.2, "mfma_flop_f16": 1e12}}},
        "gram_solve_dual_kernel<128>": {"by_grid": {"128": {
            "fetch_bytes_x2": 2e9, "write_bytes": 1e8, "pmc_run_avg_ns": 1e6, "trace_avg_ns": 1e6,
            "mfma_busy_frac": 0.2, "valu_busy_frac": 0.6, "mfma_flop_f16": 2e11}}}}}}
    monkeypatch.setattr(bench, "_pmc_doc", lambda: doc)
    parts = [("gram_solve_w1_kernel<false>", 640), ("gram_solve_dual_kernel<128>", 128)]
    c = bench._combine_pmc("w", parts)
    assert c["fetch_bytes_x2"] == 6e9 and c["trace_avg_ns"] == 4e6
    assert c["mfma_busy_frac"] == pytest.approx((0.4 * 3 + 0.2 * 1) / 4)
    assert bench._combine_pmc("w", parts + [("missing", 1)]) is None
    assert bench._combine_pmc("other", parts) is None
    r = bench.roofline("w", "k", {"user": {"ms": 4.0, "nnz": 10 ** 6, "rows": 1000, "parts": parts}},
                       128, False)
    u = r["launches"]["user"]
    assert u["pmc_profile_trace_ms"] == pytest.approx(4.0)
    assert u["mfma_issued_flops_pmc"] == pytest.approx(1.2e12)
    assert r["traffic"] == pytest.approx(6.2e9)
    assert r["frac_pmc_profile"] == pytest.approx(r["frac"])  # same duration here


@pytest.mark.parametrize("k,top,n_q,kern,grid", [
    (128, 10, 10_000_000, "topk_split_kernel<4,2,12>", 39063 * 512),
    (128, 100, 10_000_000, "topk_split_kernel<4,2,100>", 512 * 512),
    (64, 100, 162_541, "topk_split_kernel<2,1,100>", 512 * 512),
    (64, 100, 20_000, "topk_split_kernel<2,1,100>", 157 * 512),
    (64, 10, 162_541, "topk_split_kernel<2,1,12>", 1270 * 512),
    (128, 10, 262_144, "topk_split_kernel<4,2,12>", 1024 * 512),
    (128, 10, 262_143, "topk_split_kernel<4,1,12>", 2048 * 512),
    (32, 20, 1000, "topk_split_kernel<1,1,32>", 8 * 512)])
def test_topk_variant_matches_launch_choice(bench, k, top, n_q, kern, grid):
    assert bench.topk_variant(k, top, n_q) == (kern, grid)


def test_live_counter_passes_fit_the_per_pass_limits(bench):
    """Each rocprofv3 --pmc pass bench.live_counters starts stays inside gfx950's per-pass
    block limits (more in one block: 'error code 38' and a hung profiler): <= 8 SQ_,
    <= 4 TCC_ (FETCH_SIZE takes 3, WRITE_SIZE 2), <= 2 GRBM_; the kernel-trace pass carries
    no counters."""
    tcc_cost = {"FETCH_SIZE": 3, "WRITE_SIZE": 2}
    tags = [t for t, _ in bench.LIVE_PASSES]
    assert tags == ["T", "A", "B", "C", "D"]
    for tag, opts in bench.LIVE_PASSES:
        if tag == "T":
            assert opts == ["--kernel-trace"]
            continue
        assert opts[0] == "--pmc" and "--sys-trace" not in opts
        cnt = opts[1:]
        assert sum(c.startswith("SQ_") for c in cnt) <= 8
        assert sum(tcc_cost.get(c, 1 if c.startswith("TCC_") else 0) for c in cnt) <= 4
        assert sum(c.startswith("GRBM_") for c in cnt) <= 2


def test_live_counters_overlay_the_committed_profile(bench, monkeypatch):
    """Counters folded from this run's passes replace the committed entry of their
    workload only, and the roofline names where its counters came from."""
    monkeypatch.setattr(bench, "_LIVE", {"configs1": {"gram_solve_kernel<4,false>": {
        "by_grid": {"640": {"FETCH_SIZE": 1.0, "fetch_bytes_x2": 2048.0, "write_bytes": 0.0,
                            "pmc_run_avg_ns": 1000.0}}}}})
    assert bench.load_pmc("configs1", "gram_solve_kernel<4,false>", 640)["fetch_bytes_x2"] == 2048.0
    doc = bench._pmc_doc()
    assert "configs2" in doc.get("workloads", {}) or not os.path.exists(bench.PMC_FILE)
    r = bench.roofline("configs1", "gram_solve_kernel<4,false>",
                       {"item": {"ms": 1.0, "nnz": 1000, "rows": 10,
                                 "parts": [("gram_solve_kernel<4,false>", 640)]}}, 64, False)
    assert r["counters_source"].startswith("measured by this bench run")
    assert r["traffic"] == 2048.0
    r2 = bench.roofline("configs2", "gram_solve_w1_kernel<true>",
                        {"item": {"ms": 1.0, "nnz": 1000, "rows": 10,
                                  "parts": [("gram_solve_w1_kernel<true>", 640)]}}, 128, True)
    assert r2["counters_source"].startswith("profiles/pmc_summary.json")
