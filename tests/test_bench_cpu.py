"""bench.py's roofline bookkeeping on CPU: which PMC summary a workload reads
(profiles/pmc_summary.json for the match line, pmc_summary_<workload>.json for
the others), the library-hash and workload gates, and the algorithmic-byte
rescale of the config-5 superblock roofline, the device-timed roofline basis
(dispatch-inclusive with the execution span beside it) and the timed-region
kernel ranking.  No GPU call."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if not os.path.exists(mod.abi.LIB_PATH):
        pytest.skip("liblgs_hip.so not built")
    return mod


def write(path, sha, workload, kernel, fetch, write_b):
    json.dump({"lib_sha256": sha, "workload": workload,
               "kernels": {kernel: {"avg_us": 100.0, "fetch_bytes_per_launch": fetch,
                                    "write_bytes_per_launch": write_b, "l2_hit_rate": 0.5}}},
              open(path, "w"))


def test_pmc_file_per_workload(bench, tmp_path):
    sha = bench.lib_sha256()
    main = tmp_path / "pmc_summary.json"
    write(main, sha, "match", "k_coarse_list", 100, 10)
    write(tmp_path / "pmc_summary_loop.json", sha, "loop", "k_coarse_list", 40, 4)
    m = bench.pmc_for(str(main), "k_coarse_list", "match")
    assert m["traffic"] == 2 * 100 + 10 and m["raw"] == 110
    lp = bench.pmc_for(str(main), "k_coarse_list", "loop")
    assert lp["traffic"] == 2 * 40 + 4 and lp["profile"].endswith("pmc_summary_loop.json")
    assert bench.pmc_for(str(main), "k_coarse_list", "rebuild") is None      # no such file
    assert bench.pmc_for(str(main), "k_fine_lanes", "match") is None         # kernel not profiled


def test_pmc_gates(bench, tmp_path):
    main = tmp_path / "pmc_summary.json"
    write(main, "0" * 64, "match", "k_coarse_list", 100, 10)                 # another build
    assert bench.pmc_for(str(main), "k_coarse_list", "match") is None
    write(main, bench.lib_sha256(), "loop", "k_coarse_list", 100, 10)         # another workload
    assert bench.pmc_for(str(main), "k_coarse_list", "match") is None


def test_roofline_bytes_scale(bench, tmp_path):
    stats = {"k_super": dict(launches=4, total_ms=2.0, algo_bytes=4 * 8.0e9)}
    full = bench.roofline_from(stats, "k_super", str(tmp_path / "none.json"), "k_super_oct<9>", "l2-gather")
    quarter = bench.roofline_from(stats, "k_super", str(tmp_path / "none.json"), "k_super_oct<9>", "l2-gather",
                                  bytes_scale=0.25)
    assert full["achieved"] == pytest.approx(8.0e9 / 0.5e-3 / 1e9)
    assert quarter["algo_bytes_per_launch"] == pytest.approx(2.0e9)
    assert quarter["frac"] == pytest.approx(full["frac"] / 4, rel=1e-3)
    assert quarter["traffic"] is None and quarter["kernel"] == "k_super_oct<9>"
    assert bench.roofline_from({}, "k_super", "x", "k", "hbm") is None


def test_roofline_dispatch_basis_with_execution(bench, tmp_path):
    """r06 device timing: the line's roofline divides the algorithmic bytes by
    the dispatch-inclusive span and carries the execution span beside it."""
    stats = {"k_coarse": dict(launches=2, total_ms=0.4, dispatch_ms=0.5, algo_bytes=2 * 1.0e9)}
    r = bench.roofline_from(stats, "k_coarse", str(tmp_path / "none.json"), "k_coarse_list", "l2-gather",
                            time_key="dispatch_ms", exec_key="total_ms")
    assert r["time_basis"] == "dispatch_ms"
    assert r["avg_launch_ms"] == pytest.approx(0.25)
    assert r["frac"] == pytest.approx(1.0e9 / 0.25e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["execution"]["avg_launch_ms"] == pytest.approx(0.2)
    assert r["execution"]["frac"] > r["frac"]
    # without a dispatch figure (event timing) there is no dispatch roofline
    assert bench.roofline_from({"k_coarse": dict(launches=2, total_ms=0.4, dispatch_ms=0.0, algo_bytes=1e9)},
                               "k_coarse", "x", "k", "hbm", time_key="dispatch_ms") is None


def test_timed_region_ranking(bench):
    """largest_kernel: the chunk kernel with the largest share of the summed
    device-timed execution of the timed region."""
    stats = {"k_coarse": dict(launches=4, total_ms=0.8), "k_super": dict(launches=4, total_ms=1.0),
             "k_cost": dict(launches=4, total_ms=0.2), "k_unused": dict(launches=0, total_ms=0.0)}
    rows, top = bench.timed_region_kernels(stats)
    assert top["kernel"] == "k_super" and top["trace_name"] == bench.TRACE_NAMES["k_super"]
    assert top["share"] == pytest.approx(0.5) and "k_unused" not in rows
    assert rows["k_coarse"]["avg_ms"] == pytest.approx(0.2)
    assert bench.timed_region_kernels({}) == (None, None)
