"""CPU checks of the generated gfx950 butterflies (tools/gen_bfly.py ->
multilinear_amd/csrc/bfly_asm.hpp): every variant emulated lane-exactly against
big-integer arithmetic mod M (random and edge operands, rare-path flags
included), the SGPR hazard rule, the stage-twiddle precondition of the
product, and that the committed header is the generator's current output."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_bfly", os.path.join(ROOT, "tools", "gen_bfly.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("kinds", [("m", "m"), ("m",), ("t", "t"), ("t",), ("m", "t"), ("p", "p"), ("p",),
                                   ("f", "f"), ("f",), ("c", "c", "c", "c"), ("c",)])
def test_variant_emulates_exactly(kinds):
    G = _gen()
    for bsrc in (("s", "v") if any(k in ("m", "p") for k in kinds) else ("v",)):
        lines, outs, flags, ins, ns, nv, opn = G.render(kinds, bsrc)
        G.check_hazards(lines)
        assert G.selftest(kinds, lines, opn, nv, trials=1500, seed=7) == 1500 * len(kinds)


def test_rare_paths_are_reachable_and_fixed():
    """Operands that force each flag: u = v = 2^128-1 (second carry), u = 0,
    v = 2^128-1 (second borrow), w = 2 with v = 2^128-1 (product wrap)."""
    G = _gen()
    top = (1 << 128) - 1
    lines, _, _, _, _, nv, opn = G.render(("t",), "v")
    (a, d), = G.run_case(("t",), lines, opn, nv, [top], [top], [1])
    assert a % G.M == (2 * top) % G.M and d % G.M == 0
    (a, d), = G.run_case(("t",), lines, opn, nv, [0], [top], [1])
    assert a % G.M == top % G.M and d % G.M == (-top) % G.M
    lines, _, _, _, _, nv, opn = G.render(("m",), "v")
    (a, d), = G.run_case(("m",), lines, opn, nv, [5], [top], [2])
    assert a % G.M == (5 + 2 * top) % G.M and d % G.M == (5 - 2 * top) % G.M


def test_full_product_wrap_flag():
    """v * w whose folded sum carries out of 2^128 (flag K, fixed by + C):
    found by search over structured operands, e.g. (2^127 - 2) * (2^128 - 1)."""
    G = _gen()
    lines, _, _, _, _, nv, opn = G.render(("f",), "v")
    for v, w in [((1 << 127) - 2, (1 << 128) - 1), ((1 << 127) + 1, (1 << 128) - 1), (G.M - 1, G.M - 1),
                 ((1 << 128) - 1, (1 << 128) - 1), (0, G.M - 1)]:
        (_, d), = G.run_case(("f",), lines, opn, nv, [0], [v], [w])
        assert 0 <= d < (1 << 128) and d % G.M == (v * w) % G.M


def test_canonicalise_edges():
    G = _gen()
    lines, _, _, _, _, nv, opn = G.render(("c",), "v")
    for v in [0, 1, G.M - 1, G.M, G.M + 1, (1 << 128) - 1, G.C]:
        (_, d), = G.run_case(("c",), lines, opn, nv, [0], [v], [1])
        assert d == v % G.M


def test_stage_twiddle_precondition():
    assert _gen().twiddle_precondition() <= 0xFFFFFFF7


def test_header_is_current(tmp_path):
    G = _gen()
    G.OUT = str(tmp_path / "bfly_asm.hpp")
    G.main()
    committed = open(os.path.join(ROOT, "multilinear_amd", "csrc", "bfly_asm.hpp")).read()
    assert open(G.OUT).read() == committed
