"""GPU parity for the verify half: G2 setup, polyeval_G2, the optimal ate
pairing and trusted_setup::verify_proof (reference
src/trusted_setup.cpp:123-135, 176-201, 230-254), all through the C ABI.

Checker: oracle/pairing_ref.py (definitional pairing in flat Fp12 with exact
inversions and Frobenius by exponentiation -- a different algorithm from the
kernels) and the MSM-free known-tau verify of oracle/kzg_ref.py.  Every
comparison is exact: canonical G2 coordinates, the 12 canonical Fp
coefficients of the Fp12 pairing value in tower order, verify booleans."""
import numpy as np
import pytest

import kzg_ref as K
import pairing_ref as PR

pytestmark = pytest.mark.gpu

CURVES = [("BN254", K.BN254), ("BLS12381", K.BLS12381)]


def w64(C):
    return 4 if C.name == "BN254" else 6


def limbs_of(v, n):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def g1_row(C, P):
    if P is None:
        return np.zeros(2 * w64(C), dtype=np.uint64)
    return np.array(limbs_of(P[0], w64(C)) + limbs_of(P[1], w64(C)), dtype=np.uint64)


def g2_row(C, Q):
    if Q is None:
        return np.zeros(4 * w64(C), dtype=np.uint64)
    n = w64(C)
    return np.array(limbs_of(Q[0][0], n) + limbs_of(Q[0][1], n) + limbs_of(Q[1][0], n) + limbs_of(Q[1][1], n),
                    dtype=np.uint64)


def to_int(row):
    return sum(int(row[i]) << (64 * i) for i in range(len(row)))


def g2_from_row(C, row, inf=False):
    if inf:
        return None
    n = w64(C)
    v = [to_int(row[k * n:(k + 1) * n]) for k in range(4)]
    if not any(v):
        return None
    return ((v[0], v[1]), (v[2], v[3]))


def f12_row(C, f):
    out = []
    for re, im in PR.to_tower(C, f):
        out += limbs_of(re, w64(C)) + limbs_of(im, w64(C))
    return np.array(out, dtype=np.uint64)


def scalars(vals):
    return np.array([limbs_of(v % (1 << 256), 4) for v in vals], dtype=np.uint64).reshape(-1, 4)


@pytest.fixture(scope="module")
def ctxs():
    import kzgx
    made = {}

    def get(name):
        if name not in made:
            made[name] = kzgx.Context(name)
        return made[name]

    yield get
    for c in made.values():
        c.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_gen_srs_g2_matches_oracle(name, C, ctxs):
    ctx = ctxs(name)
    tau = K.default_tau(C)
    ctx.gen_srs_g2(tau, 5, start=3)
    got = ctx.get_srs_g2(5)
    ref = PR.gen_srs_g2(C, tau, 8)[3:]
    for k in range(5):
        assert g2_from_row(C, got[k]) == ref[k]
    assert ctx.g2_validate(got).all()


@pytest.mark.parametrize("name,C", CURVES)
def test_g2_validate_rejects(name, C, ctxs):
    ctx = ctxs(name)
    Q = PR.g2_generator(C)
    good = g2_row(C, Q)
    bad_y = good.copy()
    bad_y[2 * w64(C)] ^= np.uint64(1)        # y.re off by one bit -> off the twist
    big = good.copy()
    big[:w64(C)] = np.array(limbs_of(Q[0][0] + C.p, w64(C)), dtype=np.uint64) if Q[0][0] + C.p < (1 << (64 * w64(C))) \
        else big[:w64(C)]
    zero = np.zeros_like(good)
    ok = ctx.g2_validate(np.stack([good, bad_y, big, zero]))
    assert ok.tolist() == [True, False, False, False]


@pytest.mark.parametrize("name,C", CURVES)
def test_msm_g2_matches_naive(name, C, ctxs):
    ctx = ctxs(name)
    tau = K.default_tau(C)
    n = 9
    ctx.gen_srs_g2(tau, n)
    srs2 = PR.gen_srs_g2(C, tau, n)
    sc = K.random_scalars(C, n, seed=4242)
    sc[1], sc[2] = 0, C.r - 1
    out, inf = ctx.msm_g2(scalars(sc))
    assert g2_from_row(C, out, inf) == PR.polyeval_g2(C, srs2, sc)
    out, inf = ctx.msm_g2(scalars([]))       # ECP2_inf for the zero polynomial
    assert inf
    # sum that cancels to infinity: c [1]G2 + (r - c) [1]G2 via tau = 1
    ctx.gen_srs_g2(1, 2)
    out, inf = ctx.msm_g2(scalars([5, C.r - 5]))
    assert inf


@pytest.mark.parametrize("name,C", CURVES)
def test_msm_g2_windowed_edges(name, C, ctxs):
    """the windowed G2 table path: tau = 0 leaves G2[i >= 1] at infinity; scalars with
    all-zero 16-bit windows, a single set bit per window and r - 1"""
    ctx = ctxs(name)
    n = 6
    ctx.gen_srs_g2(0, n)
    srs2 = PR.gen_srs_g2(C, 0, n)
    sc = [C.r - 1, 7, 0, 1 << 200, 3, 5]
    out, inf = ctx.msm_g2(scalars(sc))
    assert g2_from_row(C, out, inf) == PR.polyeval_g2(C, srs2, sc)
    tau = K.default_tau(C)
    ctx.gen_srs_g2(tau, n)
    srs2 = PR.gen_srs_g2(C, tau, n)
    sc = [sum(1 << (16 * w + (w % 16)) for w in range(15)), (1 << 16) - 1, 1 << 240, 0, C.r - 2, 65536]
    out, inf = ctx.msm_g2(scalars(sc))
    assert g2_from_row(C, out, inf) == PR.polyeval_g2(C, srs2, sc)
    # the same SRS loaded (no tau): the table is built from the points on
    # first use (k_g2_tab) instead of from the generator's comb at setup
    # (k_g2_tab_comb); same sums
    ctx.load_srs_g2(ctx.get_srs_g2(n))
    out2, inf2 = ctx.msm_g2(scalars(sc))
    assert np.array_equal(out2, out) and inf2 == inf


@pytest.mark.parametrize("name,C", CURVES)
def test_pairing_matches_oracle(name, C, ctxs):
    ctx = ctxs(name)
    G1, G2 = (C.gx, C.gy), PR.g2_generator(C)
    a, b = 0x1234567, K.random_scalars(C, 1, seed=9)[0]
    Ps = [G1, K.scalar_mul(C, G1, a), None, G1]
    Qs = [G2, PR.g2_mul(C, G2, b), G2, None]
    got = ctx.pairing(np.stack([g1_row(C, P) for P in Ps]), np.stack([g2_row(C, Q) for Q in Qs]))
    for k in range(2):
        assert np.array_equal(got[k], f12_row(C, PR.pairing(C, Ps[k], Qs[k]))), k
    one = f12_row(C, PR.F12.one(C.p))
    assert np.array_equal(got[2], one) and np.array_equal(got[3], one)
    # bilinearity on the GPU alone: e([a]P, [b]Q) == e([a b]P, Q)
    g2 = ctx.pairing(np.stack([g1_row(C, K.scalar_mul(C, G1, a * b % C.r))]), np.stack([g2_row(C, G2)]))
    assert np.array_equal(got[1], g2[0])
    # infinity flags
    fl = ctx.pairing(np.stack([g1_row(C, G1)]), np.stack([g2_row(C, G2)]), g1_inf=[1], g2_inf=[0])
    assert np.array_equal(fl[0], one)


def _setup(ctx, C, tau, n):
    ctx.gen_srs(tau, n)
    ctx.gen_srs_g2(tau, n)


@pytest.mark.parametrize("name,C", CURVES)
def test_verify_proof_matches_reference_semantics(name, C, ctxs):
    ctx = ctxs(name)
    tau = K.default_tau(C)
    nsrs = 40
    _setup(ctx, C, tau, nsrs)
    P = K.random_scalars(C, 30, seed=31337)
    S = scalars(P)
    com, cinf = ctx.msm(S)
    cases = [(0, 1), (5, 3), (0, 29), (7, 33)]  # single, multi, deg(P)+1 > len, len > deg(P)
    for off, ln in cases:
        xs = list(range(off, off + ln))
        pts = K.evaluate_points(C, P, off, ln)
        prf, pinf = ctx.prove_range(S, scalars(xs))
        ys = [y for _, y in pts]
        ok = ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(ys))
        exp = K.verify_proof_tau(C, tau, nsrs, None if cinf else (to_int(com[:w64(C)]), to_int(com[w64(C):])),
                                 None if pinf else (to_int(prf[:w64(C)]), to_int(prf[w64(C):])), pts)
        assert ok == exp == True, (off, ln)  # noqa: E712
        bad = list(ys)
        bad[-1] = (bad[-1] + 1) % C.r
        assert not ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(bad))
    # wrong commitment
    com2, c2inf = ctx.msm(scalars(K.random_scalars(C, 30, seed=1)))
    xs, pts = [2], K.evaluate_points(C, P, 2, 1)
    prf, pinf = ctx.prove_range(S, scalars(xs))
    assert not ctx.verify_proof(com2, c2inf, prf, pinf, scalars(xs), scalars([pts[0][1]]))
    # points.size() >= |SRS| -> false (trusted_setup.cpp:235-236)
    xs = list(range(nsrs))
    assert not ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(xs))
    # empty expected data -> invalid_argument (trusted_setup.cpp:233-234)
    import kzgx
    with pytest.raises(kzgx.KzgxError):
        ctx.verify_proof(com, cinf, prf, pinf, scalars([]), scalars([]))


@pytest.mark.parametrize("name,C", CURVES)
def test_verify_proof_pairing_oracle(name, C, ctxs):
    """one case against the full pairing-form oracle (two CPU pairings)"""
    ctx = ctxs(name)
    tau = K.default_tau(C)
    nsrs = 8
    _setup(ctx, C, tau, nsrs)
    P = K.random_scalars(C, 6, seed=5)
    S = scalars(P)
    com, cinf = ctx.msm(S)
    xs = [1, 2]
    pts = K.evaluate_points(C, P, 1, 2)
    prf, pinf = ctx.prove_range(S, scalars(xs))
    s1, s2 = K.gen_srs(C, tau, nsrs), PR.gen_srs_g2(C, tau, nsrs)
    comP = (to_int(com[:w64(C)]), to_int(com[w64(C):]))
    prfP = (to_int(prf[:w64(C)]), to_int(prf[w64(C):]))
    exp = PR.verify_proof(C, s1, s2, comP, prfP, pts)
    got = ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars([y for _, y in pts]))
    assert got == exp == True  # noqa: E712


@pytest.mark.parametrize("name,C", CURVES)
def test_verify_proof_degenerate_setups(name, C, ctxs):
    """tau = 0 / 1: the identity still holds, proofs verify, tampering is caught"""
    ctx = ctxs(name)
    for tau in (1, 2):
        _setup(ctx, C, tau, 12)
        P = K.random_scalars(C, 10, seed=tau)
        S = scalars(P)
        com, cinf = ctx.msm(S)
        xs = [3, 4, 5]
        pts = K.evaluate_points(C, P, 3, 3)
        prf, pinf = ctx.prove_range(S, scalars(xs))
        ys = [y for _, y in pts]
        assert ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(ys))
        ys[0] = (ys[0] + 7) % C.r
        assert not ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(ys))


@pytest.mark.parametrize("name,C", CURVES)
def test_verify_proof_vanishing_at_tau(name, C, ctxs):
    """an opening set holding tau itself: Z(tau) = 0, so [Z(tau)]G2 is the
    point at infinity (the fused pairing kernel's Q_0 = O case: no line
    chain, e(pi, O) = 1) and the check reduces to C == [I(tau)]G1"""
    ctx = ctxs(name)
    tau = 2
    _setup(ctx, C, tau, 12)
    P = K.random_scalars(C, 10, seed=77)
    S = scalars(P)
    com, cinf = ctx.msm(S)
    xs = [2, 3, 4]
    pts = K.evaluate_points(C, P, 2, 3)
    prf, pinf = ctx.prove_range(S, scalars(xs))
    ys = [y for _, y in pts]
    exp = K.verify_proof_tau(C, tau, 12, None if cinf else (to_int(com[:w64(C)]), to_int(com[w64(C):])),
                             None if pinf else (to_int(prf[:w64(C)]), to_int(prf[w64(C):])), pts)
    assert ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(ys)) == exp == True  # noqa: E712
    for k in (0, 2):  # y at tau itself (I(tau) moves), and at another point
        bad = list(ys)
        bad[k] = (bad[k] + 1) % C.r
        bpts = [(x, y) for (x, _), y in zip(pts, bad)]
        exp = K.verify_proof_tau(C, tau, 12, None if cinf else (to_int(com[:w64(C)]), to_int(com[w64(C):])),
                                 None if pinf else (to_int(prf[:w64(C)]), to_int(prf[w64(C):])), bpts)
        assert ctx.verify_proof(com, cinf, prf, pinf, scalars(xs), scalars(bad)) == exp, k


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("wave_max", [4096, 0], ids=["wave", "lane"])
def test_verify_single_batch(name, C, ctxs, wave_max):
    """batched single-point verifies == verify_proof(commit, proof, {(z, y)})
    (reference trusted_setup.cpp:230-254 with one point), against the
    known-tau oracle on valid and tampered openings; both kernels (a wave per
    opening, a lane per opening)"""
    ctx = ctxs(name)
    ctx.set_verify_wave_max(wave_max)
    tau = K.default_tau(C)
    _setup(ctx, C, tau, 64)
    polys = [K.random_scalars(C, 40, seed=100 + i) for i in range(3)] + [[0] * 40]
    zs, ys, cs, cis, ps, pis, exp = [], [], [], [], [], [], []
    for j, P in enumerate(polys):
        S = scalars(P)
        com, cinf = ctx.msm(S)
        pts = [5, 17, C.r - 3, 0]
        prf, pinf, yv = ctx.prove_single_batch(S, scalars(pts))
        for t, z in enumerate(pts):
            y = to_int(yv[t])
            for mode in ("ok", "bad_y", "bad_z", "bad_c"):
                zz, yy, cc, ci = z, y, com, cinf
                if mode == "bad_y":
                    yy = (y + 1) % C.r
                elif mode == "bad_z":
                    zz = (z + 1) % C.r
                elif mode == "bad_c":
                    cc, ci = prf[t], pinf[t]  # a different group element in the commit slot
                zs.append(zz)
                ys.append(yy)
                cs.append(cc)
                cis.append(int(ci))
                ps.append(prf[t])
                pis.append(int(pinf[t]))
                cP = None if ci else (to_int(cc[:w64(C)]), to_int(cc[w64(C):]))
                pP = None if pinf[t] else (to_int(prf[t][:w64(C)]), to_int(prf[t][w64(C):]))
                exp.append(K.verify_proof_tau(C, tau, 64, cP, pP, [(zz, yy)]))
    got = ctx.verify_single_batch(np.stack(cs), np.stack(ps), scalars(zs), scalars(ys), commit_inf=cis,
                                  proof_inf=pis)
    assert got.tolist() == exp
    assert sum(exp) >= 16  # the valid openings (and the zero polynomial's degenerate ones)
    ctx.set_verify_wave_max(8192)
