"""tests/fixtures/cpu_calibration.json: the
restatement-vs-reference timing recorded in the build container by
tools/cpu_calibration.py.  Checks the record is present and self-consistent;
the numbers themselves are documentation for the GPU-box CPU leg."""
import json
import os

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "cpu_calibration.json")


def test_cpu_calibration_fixture():
    d = json.load(open(FIX))
    assert d["logical_cpus"] >= 1 and d["cpu_model"]
    s = d["reference_vs_restatement"]["score_pixel_accurate"]
    assert s["reference_us"] > 0 and s["restatement_us"] > 0
    assert abs(s["ratio_restatement_over_reference"] - s["restatement_us"] / s["reference_us"]) < 0.01
    # the restatement is not a handicapped port: within 2x of the reference build either way
    assert 0.5 <= s["ratio_restatement_over_reference"] <= 2.0
    o = d["oracle_config2"]
    assert o["single_scan_ms_p50"] > 0 and o["scans_per_s"] > 0 and 1 <= o["threads"] <= d["logical_cpus"]
