"""The row-bin sort network's cross-lane exchanges (csrc/lpa_lane.h: DPP quad permutes and
row rotations, gfx950 v_permlane16/32_swap, wave_shr) checked lane by lane on one wave.
The parity tests cover them through the labels; this pins the exchange itself, so a wrong
DPP control shows up as "xor j lane l" rather than as a label mismatch."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "build", "lpa_hip", "lane_xor_check")


@pytest.mark.gpu
def test_lane_exchanges_match_xor():
    if not os.path.exists(CHECK):
        pytest.fail(f"{CHECK} missing: run __graft_entry__.build() (csrc Makefile target)")
    r = subprocess.run([CHECK], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "lane_xor_check: ok" in r.stdout
