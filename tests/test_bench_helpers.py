"""bench.py's bookkeeping helpers (CPU): which profiled kernel name is the timed loop's instantiation
(the roofline's traffic, issue counters and rocprof mean must come from the kernel the headline runs),
and the strong-scaling model's arithmetic."""
import bench


def test_timed_instantiation_picks_the_headline_kernel():
    single = "k_chain<4, true, false, true, false, false, false>"
    multi = "k_chain<4, true, false, true, false, false, true>"
    counting = "k_chain<4, true, true, true, false, false, true>"
    quad = "k_chain<4, true, false, true, false, true, false>"
    assert bench.timed_instantiation("k_chain", single, multi=False)
    assert not bench.timed_instantiation("k_chain", multi, multi=False)
    assert bench.timed_instantiation("k_chain", multi, multi=True)
    assert not bench.timed_instantiation("k_chain", single, multi=True)
    assert not bench.timed_instantiation("k_chain", counting, multi=True)
    assert not bench.timed_instantiation("k_chain", quad, multi=True)
    # profiles from before the kQuad/kMulti parameters: any non-counting instantiation
    assert bench.timed_instantiation("k_chain", "k_chain<4, true, false, true, false>", multi=True)
    assert not bench.timed_instantiation("k_chain", "k_chain<4, true, true, true, false>", multi=False)
    assert bench.timed_instantiation("k_bvh_closest_hit", "k_bvh_closest_hit<4, false>", multi=False)
    assert not bench.timed_instantiation("k_chain", "k_chain_kernarg_probe", multi=False)


def test_strong_model_bounds():
    m = bench.strong_model(0.39, 0.38, 0.40, 1920 * 1080 * 3)
    for n in (2, 4, 8):
        r = m[f"n{n}"]
        assert r["render_ms"] >= 0.38 and r["render_ms"] >= 0.39 / n
        for bw in ("50GBs", "150GBs"):
            assert r[bw]["pipelined_ms_per_frame"] <= r[bw]["latency_ms_per_frame"]


def test_strong_model_takes_measured_shares():
    """With strong_shares (r06) the render and un-permute terms are the measured ones: the slowest rank's
    share one frame at a time (latency) and four frames' shares per call (pipelined)."""
    shares = {f"n{n}": {"max_ms": 0.3 / n ** 0.5, "pipelined_max_ms": 0.33 / n, "assemble_ms": 0.007} for n in (2, 4, 8)}
    m = bench.strong_model(0.36, 0.43, None, 1920 * 1080 * 3, shares=shares, t1_pipe_ms=0.323)
    assert m["inputs"]["render"].startswith("measured")
    for n in (2, 4, 8):
        r = m[f"n{n}"]
        assert r["render_ms"] == round(shares[f"n{n}"]["max_ms"], 4)
        assert r["render_pipelined_ms"] == round(shares[f"n{n}"]["pipelined_max_ms"], 4)
        assert r["assemble_ms"] == 0.007
        lat = r["150GBs"]["latency_ms_per_frame"]
        assert lat > r["render_ms"] + r["assemble_ms"]   # gather and barrier come on top
        assert abs(r["150GBs"]["pipelined_speedup"] - 0.323 / r["150GBs"]["pipelined_ms_per_frame"]) < 0.02


def test_profile_age_orders_round_tags():
    """The roofline reads the newest committed profile: round-tagged names sort by round, then by tag
    length, then by tag (r06z before r06aa: a plain string sort put r06z last and read a stale profile)."""
    names = ["r06aa_pmc.json", "r05zf_pmc.json", "r06z_pmc.json", "r06_pmc.json", "r06am_pmc.json", "r06b_pmc.json",
             "r02h_pmc.json"]
    got = sorted(names, key=bench.profile_age)
    assert got == ["r02h_pmc.json", "r05zf_pmc.json", "r06_pmc.json", "r06b_pmc.json", "r06z_pmc.json", "r06aa_pmc.json",
                   "r06am_pmc.json"]
