"""CPU: pin the oracle (oracle/combine_ref.c) against the golden vectors and
check its restated control-path rules. No GPU."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("dt", O.DTYPES)
def test_oracle_matches_golden(dt):
    z = np.load(os.path.join(GOLDEN, f"golden_{dt}.npz"))
    src, dst = z["src"], z["dst"]
    # the golden inputs are the generator's own output (after the pairs)
    tab = O.special_table(dt)
    npair = len(tab) ** 2
    base = 0x5EED0000 + 4 * O.dt_index(dt)
    assert (O.bits(src[npair:npair + 259]) == O.bits(O.fill(dt, "round", base, 259))).all()
    assert (O.bits(dst[npair + 259:]) == O.bits(O.fill(dt, "exact", base + 3, 259))).all()
    checked = 0
    for k, op in enumerate(O.OPS):
        assert bool(z["supported"][k]) == O.is_supported(dt, op)
        if not z["supported"][k]:
            with pytest.raises(ValueError):
                O.reduce(op, dt, src, dst)
            continue
        out = O.reduce(op, dt, src, dst)
        bad = np.nonzero(O.bits(out) != O.bits(z["out"][k]))[0]
        assert bad.size == 0, (op, [hex(int(O.bits(src)[i])) for i in bad[:4]])
        checked += 1
    assert checked >= 4


def test_half_conversion_matches_numpy():
    rng = np.random.default_rng(7)
    u = rng.integers(0, 2**32, size=200_000, dtype=np.uint64).astype(np.uint32)
    # add the boundary cases of RNE and overflow
    extra = np.array([0x477FF000, 0x477FEFFF, 0x477FF001, 0x33000000, 0x33000001,
                      0x387FE000, 0x387FF000, 0x38800000, 0x7F800000, 0xFF800000,
                      0x7FC00000, 0x7FC12345, 0x00000001, 0x80000000], dtype=np.uint32)
    u = np.concatenate([u, extra])
    # signalling NaNs are quieted when they cross ctypes as a C double; the
    # combine only ever rounds quiet NaNs (golden vectors cover NaN payloads)
    snan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x7FFFFF) != 0) & ((u & 0x400000) == 0)
    u = u[~snan]
    f = u.view(np.float32)
    with np.errstate(all="ignore"):
        ref = f.astype(np.float16).view(np.uint16)
    lib = O.lib()
    got = np.array([lib.ucg_oracle_float_to_half(float(x)) for x in f[:20000]],
                   dtype=np.uint16)
    got_tail = np.array([lib.ucg_oracle_float_to_half(float(x)) for x in extra.view(np.float32)],
                        dtype=np.uint16)
    # ctypes passes float through a double; NaN payloads survive that round trip
    assert (got == ref[:20000]).all()
    assert (got_tail == ref[-len(extra):]).all()
    h = np.arange(0, 2**16, dtype=np.uint32).astype(np.uint16)
    back = np.array([lib.ucg_oracle_half_to_float(int(x)) for x in h[::7]], dtype=np.float32)
    ref_b = h[::7].view(np.float16).astype(np.float32)
    nan = np.isnan(ref_b)
    assert (back[~nan].view(np.uint32) == ref_b[~nan].view(np.uint32)).all()
    assert np.isnan(back[nan]).all()


@pytest.mark.parametrize("dt", O.DTYPES)
def test_fill_is_deterministic_and_in_range(dt):
    a = O.fill(dt, "exact", 123, 4099)
    b = O.fill(dt, "exact", 123, 4099)
    c = O.fill(dt, "exact", 124, 4099)
    assert (O.bits(a) == O.bits(b)).all()
    assert (O.bits(a) != O.bits(c)).any()
    if dt in ("float32", "float64", "float16"):
        assert np.all(np.abs(a.astype(np.float64)) <= 1024)
        assert np.all(a.astype(np.float64) == np.round(a.astype(np.float64)))
    sp = O.fill(dt, "special", 5, 2000)
    table = set(O.special_table(dt))
    assert set(int(x) for x in O.bits(sp)) <= table


def test_fragment_rule():
    # builtin/ops/builtin_control.c:434,462-465
    assert O.frag_length(256, 4) == 248
    assert O.frag_length(256, 8) == 248
    assert O.frag_length(2048, 8) == 2040
    assert O.frag_length(100, 12) == 84
    assert O.fragments_total(4096, 248, 1) == 17
    assert O.fragments_total(4096, 248, 3) == 51
    assert O.fragments_total(248 * 4, 248, 1) == 4


def test_recursive_peer_is_xor():
    # builtin/plan/builtin_recursive.c:162-169 with factor 2
    for size in (2, 4, 8, 16, 64):
        steps = size.bit_length() - 1
        for my in range(size):
            for step in range(1, steps + 1):
                assert O.recursive_peer(my, step) == my ^ (1 << (step - 1))


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16])
def test_reduce_multi_integers_equal_plain_sum(n):
    srcs = [O.fill("int64", "round", 1000 + r, 333) for r in range(n)]
    want = np.zeros(333, dtype=np.uint64)
    for s in srcs:
        want += s.view(np.uint64)
    for self_index in range(n):
        got = O.reduce_multi("sum", "int64", srcs, self_index)
        assert (got.view(np.uint64) == want).all()


def test_reduce_multi_float_is_recursive_doubling_tree():
    # exact association ((x0+x1)+(x2+x3)) as seen from member 0, and member 3
    # computes ((x2+x3)+(x0+x1)) with its own subtree as the dst operand
    xs = [O.fill("float32", "round", 77 + r, 1001) for r in range(4)]
    r0 = O.reduce_multi("sum", "float32", xs, 0)
    with np.errstate(all="ignore"):
        t = (xs[1] + xs[0]) + (xs[3] + xs[2])
    assert (r0.view(np.uint32) == t.view(np.uint32)).all()


def test_fragmented_equals_whole_for_elementwise():
    s = O.fill("float64", "round", 1, 10_001)
    d = O.fill("float64", "round", 2, 10_001)
    a = O.reduce("sum", "float64", s, d)
    b = O.reduce("sum", "float64", s, d, frag_bytes=O.frag_length(256, 8))
    assert (a.view(np.uint64) == b.view(np.uint64)).all()


def test_mpich_callback_bench_agrees_with_oracle():
    """oracle/_build/mpich_bench times MPI_Reduce_local - the combine the
    reference calls through reduce_cb_f - for bench.py's CPU baseline; its
    whole-buffer result must equal the oracle's bit for bit (it exits 3
    otherwise). Skipped where MPICH is absent."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "oracle", "_build", "mpich_bench")
    if not os.path.exists(exe):
        pytest.skip("MPICH not present: mpich_bench not built")
    p = subprocess.run([exe, str(100_003), "0.2", "256"], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["bit_exact_vs_oracle"] is True and res["fragment_bytes"] == 248
