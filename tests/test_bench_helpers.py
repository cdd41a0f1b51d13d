"""CPU checks of bench.py's measurement arithmetic (no GPU): the SQ-pass figures (VALU-busy
fraction, wave-cycle split) and the limiter that sets roofline.bound from them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_sq_fields_round3_profile():
    """The round-3 sponza PMC pass (profiles/r03_r03r_summary.md, one launch): 6,144 waves,
    1,051.2e9 wave quad-cycles, 227.4e9 VALU instructions -> the 0.34 / 0.39 / 0.27 split and
    VALU pipes busy ~0.65 of the launch."""
    agg = {"SQ_WAVES": 6144.0, "SQ_WAVE_CYCLES": 1051221112734.0, "SQ_WAIT_ANY": 407607722278.0,
           "SQ_WAIT_INST_ANY": 285739843156.0, "SQ_ACTIVE_INST_ANY": 357873547300.0,
           "SQ_INSTS_VALU": 227429489776.0}
    sq = bench.sq_fields(agg, 1)
    ws = sq["wave_split"]
    assert (ws["issuing"], ws["waiting"], ws["issue_stalled"]) == (0.3404, 0.3877, 0.2718)
    launch_cycles = 4 * 1051221112734.0 / 6144
    assert abs(sq["valu_busy"] - 227429489776.0 * 2 / (1024 * launch_cycles)) < 1e-4
    assert 0.6 < sq["valu_busy"] < 0.7
    # two launches aggregated: the same per-launch figures
    sq2 = bench.sq_fields({k: 2 * v for k, v in agg.items()}, 2)
    assert sq2["valu_busy"] == sq["valu_busy"] and sq2["wave_split"] == ws
    assert bench.sq_fields({}, 1) is None


def test_sq_fields_grid_waves_round5_bunny():
    """Round 5's bunny pass (one dispatch of a 6,144-wave persistent grid): SQ_WAVES read 12,288,
    SQ_WAVE_CYCLES 357.3e9 quad-cycles, SQ_INSTS_VALU 84.8e9.  Taken from the grid, the launch
    length gives VALU pipes busy ~0.71 (round 4's figure); from SQ_WAVES it read 1.42, an
    impossible fraction.  SQ_WAVES is kept in `raw`."""
    agg = {"SQ_WAVES": 12288.0, "SQ_WAVE_CYCLES": 357326536227.0, "SQ_INSTS_VALU": 84808015695.0,
           "SQ_WAIT_ANY": 0.32 * 357326536227.0, "SQ_WAIT_INST_ANY": 0.3268 * 357326536227.0,
           "SQ_ACTIVE_INST_ANY": 0.3532 * 357326536227.0}
    sq = bench.sq_fields(agg, 1, grid_waves=6144)
    assert 0.70 < sq["valu_busy"] < 0.72
    assert sq["raw"]["SQ_WAVES"] == 12288.0 and sq["raw"]["grid_waves"] == 6144.0
    assert bench.sq_fields(agg, 1)["valu_busy"] > 1.0  # the SQ_WAVES form


def test_limiter():
    assert bench.limiter(0.8, None) == "hbm"
    assert bench.limiter(0.375, {"valu_busy": 0.75}) == "valu"
    assert bench.limiter(0.375, {"valu_busy": 0.65}) == "latency"
    assert bench.limiter(None, None) == "unmeasured"


def test_dominant_kernel_names():
    """The rocprof kernel names bench.py matches its PMC rows against (k_render_ps's template
    arguments <STATS, COST, CN, W, TRIS, PK>)."""
    assert bench.dominant_kernel(1, 6) == "wgt::k_render_ps<false, false, 1, 6, true, true>"
    assert bench.dominant_kernel(0, 5, park=False) == "wgt::k_render_ps<false, false, 0, 5, true, false>"
    assert bench.dominant_kernel(1, 6, tris=False) == "wgt::k_render_ps<false, false, 0, 8, false, false>"


def test_node_form_from_scene_info():
    """The node form comes from the library's scene_info (0 = 128-B nodes, 1 = 80-B compact)."""
    assert bench.node_form({"node_form": 1, "ps_waves": 6}) == 1
    assert bench.node_form({"node_form": 0, "ps_waves": 5}) == 0
