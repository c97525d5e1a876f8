"""The static DPP-hazard check that guards the two-lane SHA-256's inline-asm
DPP (tools/dpp_hazard_check.py; the Makefile runs it on every link): the
walk-back rule on synthetic listings, and the built library clean."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dpp_hazard_check as H  # noqa: E402

HDR = "0000000000001000 <kern>:"
DPP = "\tv_add_u32_dpp v6, v5, v7 row_half_mirror row_mask:0xf bank_mask:0x5 // 000000001010: 0"


def test_walk_back_rule():
    hit = [HDR, "\tv_add_u32_e32 v5, v1, v2 // 0", DPP]
    assert H.check_listing(hit)[1], "a write just before the DPP source is a hazard"
    one = [HDR, "\tv_add_u32_e32 v5, v1, v2 // 0", "\tv_xor_b32_e32 v9, v1, v2 // 0", DPP]
    assert H.check_listing(one)[1], "one wait state is not enough"
    two = [HDR, "\tv_add_u32_e32 v5, v1, v2 // 0", "\tv_xor_b32_e32 v9, v1, v2 // 0",
           "\tv_xor_b32_e32 v8, v1, v2 // 0", DPP]
    assert not H.check_listing(two)[1]
    nop = [HDR, "\tv_add_u32_e32 v5, v1, v2 // 0", "\ts_nop 1 // 0", DPP]
    assert not H.check_listing(nop)[1]
    pair = [HDR, "\tv_mad_u64_u32 v[4:5], s[0:1], v1, v2, 0 // 0", DPP]
    assert H.check_listing(pair)[1], "a 64-bit destination covering the source"
    other = [HDR, "\tv_add_u32_e32 v4, v1, v2 // 0", DPP]
    assert H.check_listing(other) == (1, [])


def test_built_library_has_no_dpp_hazard():
    lib = os.path.join(ROOT, "multilinear_amd", "libmlhip.so")
    if not os.path.exists(lib):
        pytest.skip("libmlhip.so not built")
    assert H.main([lib]) == 0
