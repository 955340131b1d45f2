"""bench.py host logic that runs without a GPU (the final JSON must never fail after the timed legs)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pmc_traffic_every_arithmetic():
    b = _bench()
    for math in b.CONV_MATH_INFO:
        v = b.pmc_traffic(math)
        assert v is None or (isinstance(v, int) and v > 0), (math, v)
    # h3 has a FETCH_SIZE / WRITE_SIZE pass of the halo kernel: calibrated bytes, ~1.0-1.1x the 1.07 GB algorithmic
    h3 = b.pmc_traffic("h3")
    assert h3 is not None and 0.9e9 < h3 < 1.5e9


def test_pmc_traffic_missing_keys(tmp_path, monkeypatch):
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r9_pmc_conv128_x6.json").write_text('{"kernel": "x"}')
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    assert b.pmc_traffic("x6") is None
    (prof / "r9_pmc_conv128.json").write_text('{"traffic_bytes": 1234}')
    assert b.pmc_traffic("fp32") == 1234
    (prof / "r9_pmc_conv128_h3.json").write_text('{"FETCH_SIZE": 10, "WRITE_SIZE": 2}')
    assert b.pmc_traffic("h3") == int((10 / b.HALO_FETCH_PER_BYTE + 2) * 1024)
