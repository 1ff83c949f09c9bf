"""The round-6 measurement tools on CPU: the float-model divergence study (oracle only) and the
short-launch attribution (over a synthetic stamped timeline with a known answer)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_float_model_divergence_small(tmp_path, oracle_lib):
    """STRICT32 vs DOUBLE on a small slice of C3's stream: positions part (the models differ on a few %
    of single movement updates), the discrete outputs of the first ticks agree, and the
    report's fractions are consistent with each other."""
    out = tmp_path / "div.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "float_model_divergence.py"), "--envs", "512",
                        "--ticks", "150", "--every", "50", "--out", str(out)], cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(out.read_text())
    assert d["envs"] == 512 and d["ticks"] == 150 and len(d["series"]) == 3
    assert 0.0 < d["arenas_ever_differed"] <= 1.0
    assert d["arenas_outputs_ever_differed"] <= d["arenas_ever_differed"] + 1e-12
    assert d["arenas_discrete_outputs_ever_differed"] <= d["arenas_outputs_ever_differed"]
    assert d["first_tick_each_output_field_differed"].get("position") is not None
    assert 0.0 < d["max_abs_position_difference"]
    for row in d["series"]:
        assert row["discrete_outputs_differ"] <= row["outputs_differ"] <= 1.0


def test_short_launch_attribution_known_answer():
    """A synthetic timeline (100 MHz stamps): two waves of a 20-tick launch and the 1000-tick
    reference.  The critical path is the wave that drains last, and its parts sum to the span."""
    import short_launch_attribution as sla

    def wave(t0, pro, loop, drain, slot):
        return [t0, t0 + pro, t0 + pro + loop, t0 + pro + loop + drain, slot, 3]
    doc = {"raw_20": [wave(0, 80, 1900, 20, 0), wave(50, 90, 2100, 30, 1)],
           "raw_1000": [wave(0, 100, 90000, 20, 0), wave(0, 100, 92000, 20, 1)]}
    a = sla.analyse(doc, 20)
    cp = a["critical_path"]
    assert a["span_us"] == 22.7  # (50 + 90 + 2100 + 30) / 100
    assert cp["dispatch_stagger_us"] == 0.5 and cp["prologue_us"] == 0.9 and cp["drain_us"] == 0.3
    assert cp["steady_ticks_us"] == 18.2  # 20 x the 1000-tick median (910 us / 1000)
    assert abs(cp["loop_ramp_us"] - (20.0 - 18.2)) < 1e-9 and abs(cp["loop_tail_us"] - 1.0) < 1e-9
    assert abs(a["check_sum_us"] - a["span_us"]) < 1e-6
    assert a["last_wave"]["slot"] == 1 and a["last_wave"]["xcc"] == 3
