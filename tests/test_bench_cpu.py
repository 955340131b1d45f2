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


def test_whole_path_rooflines_and_step_stats():
    """The bench line's whole-path fractions (north_star: train-step and T=1500 sampling throughput as roofline
    fractions) and the median step, on round 5's driver numbers: C2 47.988 ms per 256-image step ->
    0.368 of the h3 ceiling; sampling 12.961 ms per denoise step at n = 256 -> 0.455; a CFG step runs 2n images."""
    b = _bench()
    wp = b.whole_path_rooflines("h3", 256, 47.988, 256, {"w=0": 12.961, "w=3": 25.0})
    assert abs(wp["train_step"]["frac"] - 0.3682) < 2e-3
    assert abs(wp["sample_w=0"]["frac"] - 0.4546) < 2e-3
    assert wp["sample_w=3"]["forward_images_per_step"] == 512
    assert abs(wp["sample_w=3"]["achieved"] - 2 * wp["sample_w=0"]["achieved"] * 12.961 / 25.0) < 0.05
    assert wp["train_step"]["peak"] == round(2500.0 / 3, 2)
    c4 = b.whole_path_rooflines("bf16", 256, 26.408, 256, {"w=0": 7.0})
    assert c4["train_step"]["peak"] == 2500.0 and abs(c4["train_step"]["frac"] - 0.2231) < 2e-3
    st = b.step_stats([3.0, 1.0, 2.0, 10.0])
    assert st["median_ms"] == 2.5 and st["min_ms"] == 1.0 and st["max_ms"] == 10.0 and st["steps"] == 4
    assert b.step_stats([4.0, 1.0, 2.0])["median_ms"] == 2.0
    assert b.step_stats([]) is None


def _run_bench(*args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` (the driver's command shape, no rank environment) starts 2 ranks itself and relays rank 0's
    single JSON line: n_gpus 2, parallelism dp2 (VERDICT r4 missing-1).  CPU rehearsal: --plumbing-check (gloo)."""
    rc, lines, err = _run_bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--plumbing-check")
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 512
    assert out["plumbing_only"] is True and out["value"] is None


def test_bench_world_size_mismatch_fails():
    """A rank environment that disagrees with --gpus exits non-zero instead of measuring the wrong world."""
    rc, lines, _ = _run_bench("--gpus", "2", "--steps", "1", "--warmup", "0", "--plumbing-check",
                              env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines
