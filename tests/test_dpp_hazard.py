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
    other = [HDR, "\ts_nop 1 // 0", "\tv_add_u32_e32 v4, v1, v2 // 0", DPP]
    assert H.check_listing(other) == (1, [])


def _ins(addr, text):
    return "\t%s // %012X: 0" % (text, addr)


def test_block_entries_and_exec_rule():
    """A DPP at a branch target, at the function entry or right after a call
    return has predecessors the walk cannot see: reported unless an s_nop
    already covers the wait states.  A VALU EXEC write (v_cmpx, or an exec
    destination) needs 5 wait states before a DPP."""
    hdr = "0000000000001000 <kern>:"
    dpp = "v_add_u32_dpp v6, v5, v7 row_half_mirror row_mask:0xf bank_mask:0x5"
    br = "s_cbranch_scc1 2 // 000000001000: BF850002 <kern+0x10>"
    # branch to 0x1010 (the DPP's own address): the taken path's predecessor is unseen
    at_target = [hdr, "\t" + br, _ins(0x1004, "v_xor_b32_e32 v9, v1, v2"),
                 _ins(0x1008, "v_xor_b32_e32 v8, v1, v2"), _ins(0x100C, "v_xor_b32_e32 v7, v1, v2"),
                 _ins(0x1010, dpp)]
    assert H.check_listing(at_target)[1], "DPP at a branch target"
    covered = [hdr, "\t" + br, _ins(0x1004, "v_xor_b32_e32 v9, v1, v2"),
               _ins(0x1008, "v_xor_b32_e32 v8, v1, v2"), _ins(0x100C, "v_xor_b32_e32 v7, v1, v2"),
               _ins(0x1010, "s_nop 1"), _ins(0x1014, dpp)]
    # (the target is now the s_nop: 2 wait states covered before the entry is reached)
    covered[1] = "\ts_cbranch_scc1 3 // 000000001000: BF850003 <kern+0x10>"
    assert not H.check_listing(covered)[1]
    entry = [hdr, _ins(0x1000, dpp)]
    assert H.check_listing(entry)[1], "DPP as the first instruction of a function"
    call = [hdr, _ins(0x1000, "v_xor_b32_e32 v9, v1, v2"), _ins(0x1004, "v_xor_b32_e32 v8, v1, v2"),
            _ins(0x1008, "s_swappc_b64 s[30:31], s[4:5]"), _ins(0x100C, dpp)]
    assert H.check_listing(call)[1], "DPP right after a call returns"
    pad = ["v_xor_b32_e32 v%d, v1, v2" % r for r in (20, 21, 22, 23, 24)]
    cmpx = [hdr] + [_ins(0x1000 + 4 * i, t) for i, t in
                    enumerate(pad + ["v_cmpx_eq_u32_e32 vcc, v1, v2", pad[0], pad[1], dpp])]
    assert H.check_listing(cmpx)[1], "v_cmpx 2 wait states before a DPP"
    far = [hdr] + [_ins(0x1000 + 4 * i, t) for i, t in
                   enumerate(pad + ["v_cmpx_eq_u32_e32 vcc, v1, v2"] + pad + [dpp])]
    assert not H.check_listing(far)[1], "5 wait states cover an EXEC write"
    ex = [hdr] + [_ins(0x1000 + 4 * i, t) for i, t in
                  enumerate(pad + ["v_cmp_eq_u32_e64 exec, v1, v2", pad[0], dpp])]
    assert H.check_listing(ex)[1], "VALU with an exec destination"


def test_built_library_has_no_dpp_hazard():
    lib = os.path.join(ROOT, "multilinear_amd", "libmlhip.so")
    if not os.path.exists(lib):
        pytest.skip("libmlhip.so not built")
    assert H.main([lib]) == 0
